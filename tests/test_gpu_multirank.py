"""The product path multi-rank: bench.py and ``python -m ldpc_amd.sweep`` as 2 ranks with the HIP decoder
in the loop.  Each rank is a FRESH child process (subprocess; the test process never execs); both share
cuda:0 (LDPC_BENCH_SHARE_GPU) and reduce their counters over gloo (LDPC_BENCH_BACKEND) — on the driver's
8-GPU node the same code runs one GPU per rank over RCCL.  This covers what the oracle-decoded gloo test
(test_dist.py) cannot: the rank-offset LLR generation (``rank * B`` into ldpc_random_bits /
ldpc_awgn_llr), ``max_over_ranks`` and the counter all-reduce of device tensors.  The union of the two
shards is the same data as one process decoding both, so the summed counts must be EQUAL.
Reference multi-GPU mode: nn.DataParallel, pytorch/ofdm/ofdm_functions.py:141-145."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(args, world, timeout=240):
    """Start ``world`` ranks of ``python <args>`` as child processes; return rank 0's stdout."""
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LDPC_BENCH_SHARE_GPU="1",
                   LDPC_BENCH_BACKEND="gloo", PYTHONPATH=os.path.join(ROOT, "ldpc-sims_amd"))
        if world == 1:
            for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_PORT"):
                env.pop(k)
        procs.append(subprocess.Popen([sys.executable, *args], cwd=ROOT, env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    try:
        for p in procs:
            o, e = p.communicate(timeout=timeout)
            assert p.returncode == 0, e[-3000:]
            outs.append(o)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return outs[0]


def _bench_line(out):
    return json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])


def test_bench_two_ranks_equal_one_process_over_both_shards():
    common = ["bench.py", "--steps", "2", "--warmup", "1", "--iters", "10", "--ebn0", "1:1:3",
              "--no-cpu-baseline", "--no-legs"]
    two = _bench_line(_launch([*common, "--gpus", "2", "--batch", "4096"], 2))
    one = _bench_line(_launch([*common, "--gpus", "1", "--batch", "8192"], 1))
    assert two["n_gpus"] == 2 and two["config"]["global_batch"] == 8192 and two["value"] > 0
    rk = two["ranks"]   # what the process group itself reports, gathered over it
    assert rk["world_size"] == 2 and rk["backend"] == "gloo" and [r["rank"] for r in rk["per_rank"]] == [0, 1]
    assert one["ranks"]["world_size"] == 1
    assert two["ber"]["codewords_per_point"] == one["ber"]["codewords_per_point"] == 8192
    assert two["ber"]["coded_ber_info"] == one["ber"]["coded_ber_info"]
    assert two["ber"]["coded_bler"] == one["ber"]["coded_bler"]
    assert 0 < one["ber"]["coded_bler"][0] < 1   # a point with errors, so equal counts mean something


def test_bench_gpus2_starts_its_own_ranks():
    """``python bench.py --gpus 2`` with NO launcher variables (the driver's plain invocation): bench.py
    starts the two rank processes itself (ldpc_amd.dist.spawn_ranks) before touching the GPU; the line
    reports 2 GPUs, the process group saw world size 2, and the counts equal one process over both shards.
    (Shared-GPU / gloo rehearsal switches only because this box has one GPU.)"""
    common = ["bench.py", "--steps", "2", "--warmup", "1", "--iters", "10", "--ebn0", "1:1:3",
              "--no-cpu-baseline", "--no-legs"]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE",
                                                              "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(LDPC_BENCH_SHARE_GPU="1", LDPC_BENCH_BACKEND="gloo", PYTHONPATH=os.path.join(ROOT, "ldpc-sims_amd"))
    p = subprocess.run([sys.executable, *common, "--gpus", "2", "--batch", "4096"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1                                   # rank 0's line only
    two = json.loads(lines[0])
    one = _bench_line(_launch([*common, "--gpus", "1", "--batch", "8192"], 1))
    assert two["n_gpus"] == 2 and two["ranks"]["world_size"] == 2 and two["config"]["global_batch"] == 8192
    assert [r["rank"] for r in two["ranks"]["per_rank"]] == [0, 1]
    assert two["ber"] == one["ber"]


def test_sweep_two_ranks_equal_one_process(tmp_path):
    common = ["-m", "ldpc_amd.sweep", "--code", "wifi648_12", "--algo", "minsum", "--iters", "10",
              "--snr", "1:1:3", "--n", "10000", "--batch", "3000", "--seed", "4"]
    _launch([*common, "--out", str(tmp_path / "two.json")], 2)
    _launch([*common, "--out", str(tmp_path / "one.json")], 1)
    # --gpus 2 without launcher variables: the sweep starts its own two ranks
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE",
                                                              "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(LDPC_BENCH_SHARE_GPU="1", LDPC_BENCH_BACKEND="gloo", PYTHONPATH=os.path.join(ROOT, "ldpc-sims_amd"))
    p = subprocess.run([sys.executable, *common, "--gpus", "2", "--out", str(tmp_path / "own.json")], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    two = json.load(open(tmp_path / "two.json"))
    one = json.load(open(tmp_path / "one.json"))
    own = json.load(open(tmp_path / "own.json"))
    assert two["codewords"] == one["codewords"] == own["codewords"] == [10000] * 3
    for key in ("uncoded_ber", "coded_ber", "coded_bler"):
        assert two[key] == one[key] == own[key], key


def test_bench_dvbs2_config4_two_ranks_equal_one_process():
    """BASELINE config [4]'s sharded leg on its own code: DVB-S2 (EN 302 307) 64800 rate 1/2, 50 min-sum
    iterations, the batch sharded over 2 ranks (256 codewords each) with the counter all-reduce — summed
    counts equal one process decoding both shards (the reference's multi-GPU mode it replaces:
    nn.DataParallel, ofdm_functions.py:141-145)."""
    common = ["bench.py", "--code", "dvbs2_12", "--iters", "50", "--steps", "1", "--warmup", "0",
              "--ebn0", "1.2:0.2:1.6", "--no-cpu-baseline", "--no-dropin"]
    two = _bench_line(_launch([*common, "--gpus", "2", "--batch", "256"], 2, timeout=400))
    one = _bench_line(_launch([*common, "--gpus", "1", "--batch", "512"], 1, timeout=400))
    assert two["ranks"]["world_size"] == 2 and two["config"]["global_batch"] == 512
    assert two["config"]["kernel_path"] == "ira-z360" and two["config"]["iters"] == 50
    assert two["ber"]["codewords_per_point"] == one["ber"]["codewords_per_point"] == 512
    assert two["ber"]["coded_ber_info"] == one["ber"]["coded_ber_info"]
    assert two["ber"]["coded_bler"] == one["ber"]["coded_bler"]
    assert one["ber"]["coded_bler"][0] > 0 and one["ber"]["coded_bler"][-1] < one["ber"]["coded_bler"][0]


def test_bench_multigpu_runs_the_config4_leg():
    """At N>1 bench.py also runs BASELINE config [4] (DVB-S2 64800 rate 1/2, 50 min-sum iterations) on every
    rank — the multi-GPU configuration BASELINE names — under side.configs.config4, with max-over-ranks
    timing, every rank's timed seconds in its ``ranks`` and the counters summed by the all-reduce: equal to
    one process decoding both shards (here 256 codewords per rank through --leg-batch-scale)."""
    common = ["bench.py", "--steps", "1", "--warmup", "0", "--iters", "5", "--batch", "1024", "--ebn0", "1:1:2",
              "--no-cpu-baseline", "--no-dropin"]
    two = _bench_line(_launch([*common, "--gpus", "2", "--leg-batch-scale", "0.0625"], 2, timeout=400))
    one = _bench_line(_launch([*common, "--gpus", "1", "--legs", "config4", "--leg-batch-scale", "0.125"], 1,
                              timeout=400))
    l2, l1 = two["side"]["configs"]["config4"], one["side"]["configs"]["config4"]
    assert list(two["side"]["configs"]) == ["config4"] and list(one["side"]["configs"]) == ["config4"]
    assert l2["n_gpus"] == 2 and l2["config"]["code"] == "dvbs2_12" and l2["config"]["iters"] == 50
    assert l2["config"]["batch_per_gpu"] == 256 and l2["config"]["global_batch"] == 512
    assert l2["config"]["kernel_path"] == "ira-z360"
    rk = l2["ranks"]
    assert rk["world_size"] == 2 and [r["rank"] for r in rk["per_rank"]] == [0, 1]
    assert all(r["timed_s"] > 0 for r in rk["per_rank"])
    assert abs(l2["value"] - 2 * l2["steps"] * 256 / (l2["ms_per_step"] * l2["steps"] / 1e3)) <= 1e-6 * l2["value"]
    assert l2["ber"]["codewords_per_point"] == l1["ber"]["codewords_per_point"] == 512
    assert l2["ber"]["coded_ber_info"] == l1["ber"]["coded_ber_info"]
    assert l2["ber"]["coded_bler"] == l1["ber"]["coded_bler"]
    assert l2["roofline"]["bound"].startswith("memory-side") and l2["roofline"]["frac"] > 0  # IRA: Infinity-Cache bytes


def test_bench_rccl_process_group_on_one_gpu():
    """The RCCL path itself on the real device: bench.py under a process group with the default backend
    ("nccl" = RCCL) at world size 1 (LDPC_BENCH_PG=1; RCCL refuses two ranks on one GPU — "Duplicate GPU
    detected", scripts/rccl_probe.py — so the 2-rank tests above reduce over gloo).  The group initialises
    with the decode device, the timed region's barriers and the rank gather run over RCCL, and the record
    reports backend nccl with this GPU; the counts equal a run without a process group."""
    common = ["bench.py", "--steps", "2", "--warmup", "1", "--iters", "10", "--ebn0", "1:1:3", "--batch", "4096",
              "--no-cpu-baseline", "--no-legs", "--no-dropin"]
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", LOCAL_WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()), LDPC_BENCH_PG="1", PYTHONPATH=os.path.join(ROOT, "ldpc-sims_amd"))
    for k in ("LDPC_BENCH_BACKEND", "LDPC_BENCH_SHARE_GPU"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, *common], cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    pg = _bench_line(p.stdout)
    plain = _bench_line(_launch(common, 1))
    rk = pg["ranks"]
    assert rk["world_size"] == 1 and rk["backend"] == "nccl" and rk["per_rank"][0]["rank"] == 0
    assert rk["per_rank"][0]["name"] == plain["ranks"]["per_rank"][0]["name"]
    assert plain["ranks"]["backend"] is None
    assert pg["ber"] == plain["ber"] and pg["value"] > 0
