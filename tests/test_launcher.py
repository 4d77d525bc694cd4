"""``--gpus N`` is authoritative: bench.py / ``ldpc_amd.sweep`` start N rank processes
themselves when no launcher did (``ldpc_amd.dist.spawn_ranks``), and refuse a launcher whose WORLD_SIZE
differs from N.  Here on CPU with gloo ranks; tests/test_gpu_multirank.py runs ``bench.py --gpus 2`` with
the HIP decoder.  Reference multi-GPU mode it replaces: nn.DataParallel, ofdm_functions.py:141-145."""
import json
import os
import subprocess
import sys
import time

import pytest

from ldpc_amd.dist import RANK_VARS, resolve_world, spawn_ranks

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "launch_worker.py")


def _clean_env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in RANK_VARS}
    env.update(extra)
    return env


def test_resolve_world():
    assert resolve_world(1, {}) == 1
    assert resolve_world(8, {}) == 8
    assert resolve_world(2, {"WORLD_SIZE": "2"}) is None      # one rank of an existing launch
    with pytest.raises(SystemExit, match="WORLD_SIZE=4"):
        resolve_world(2, {"WORLD_SIZE": "4"})
    with pytest.raises(SystemExit):
        resolve_world(0, {})


def test_spawn_ranks_gloo(capfd):
    rc = spawn_ranks([WORKER], 3, env=_clean_env())
    assert rc == 0
    line = [x for x in capfd.readouterr().out.splitlines() if x.startswith("{")]
    assert len(line) == 1                                      # rank 0 only
    rec = json.loads(line[0])
    assert rec == {"world": 3, "sum": 6, "local": "0", "addr": "127.0.0.1"}


def test_spawn_ranks_failure_ends_the_others():
    """Rank 1 fails before the collective; rank 0 and 2 would wait in it forever: the launcher ends them and
    returns rank 1's code."""
    t = time.perf_counter()
    rc = spawn_ranks([WORKER, "--fail-rank", "1"], 3, env=_clean_env())
    assert rc == 3
    assert time.perf_counter() - t < 60


@pytest.mark.parametrize("script", ["bench.py", "sweep"])
def test_world_size_mismatch_refused(script):
    cmd = [sys.executable, "bench.py", "--gpus", "1"] if script == "bench.py" else \
        [sys.executable, "-m", "ldpc_amd.sweep", "--gpus", "1"]
    env = _clean_env(WORLD_SIZE="2", RANK="0", PYTHONPATH=os.path.join(ROOT, "ldpc-sims_amd"))
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "WORLD_SIZE=2" in p.stderr and "--gpus 1" in p.stderr


def test_bench_refuses_more_gpus_than_visible():
    """Without the shared-GPU rehearsal switch, --gpus N needs N visible devices (none in this container)."""
    env = _clean_env(PYTHONPATH=os.path.join(ROOT, "ldpc-sims_amd"))
    env.pop("LDPC_BENCH_SHARE_GPU", None)
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2"], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=120)
    assert p.returncode != 0 and "--gpus 2 but only" in p.stderr
