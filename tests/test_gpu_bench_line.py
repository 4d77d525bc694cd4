"""The bench.py JSON line (the driver's contract, BASELINE.json metric) on a short run: every field the
round's records rely on is present and consistent — the value from the step time, the roofline with its
counters, the CPU baselines (the C port timed here and the reference's own CPU record, never silently
dropped), the side measurements, the rank evidence and the BER curve."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_line_contract():
    out = subprocess.run([sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--batch", "8192",
                          "--cpu-seconds", "0.5", "--leg-batch-scale", "0.0625"], cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["metric"] == json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
    assert d["unit"] == "codewords/s" and d["higher_is_better"] is True and d["n_gpus"] == 1
    assert abs(d["value"] - 8192 / (d["ms_per_step"] / 1e3)) <= 1e-6 * d["value"]
    roof = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in roof
    assert roof["bound"] in ("lds", "valu", "hbm") and roof["frac"] > 0
    cpu = d["cpu_baseline"]
    assert cpu["kind"] == "port" and cpu["value"] > 0 and cpu["cores"] >= 1
    ref = cpu["reference"]
    assert ref["kind"] == "reference" and "missing" not in ref, ref
    assert ref["value"] > 0 and ref["gpu_tanh_sp_over_reference"] > 1e5 and ref["dropin_over_reference"] > 1e4
    assert d["side"]["gpu_tanh_sp"]["cw_per_s"] > 0 and d["dropin_cw_per_s"] > 0
    assert d["ranks"]["world_size"] == 1 and len(d["ranks"]["per_rank"]) == 1
    assert len(d["ber"]["ebn0_db"]) == 11 and d["ber"]["codewords_per_point"] == 8192
    assert d["side"]["gpu_tanh_sp"]["timing"] == "HIP events" and d["side"]["gpu_tanh_sp"]["launches"] >= 20
    # BASELINE configs[2..4] as side legs (never `value`), each event-timed with its own roofline
    legs = d["side"]["configs"]
    assert sorted(legs) == ["config2", "config3", "config4"]
    want = {"config2": ("wifi1944_56", "tanh", 50, "16qam-ofdm", False, 2048),
            "config3": ("wifi1296_23", "qminsum", 20, "bpsk", True, 4096),
            "config4": ("dvbs2_12", "minsum", 50, "bpsk", False, 256)}
    for name, (code, algo, iters, mod, es, b) in want.items():
        lg = legs[name]
        c = lg["config"]
        assert (c["code"], c["algo"], c["iters"], c["mod"], c["early_stop"], c["batch_per_gpu"]) == \
            (code, algo, iters, mod, es, b), name
        P = len(lg["ber"]["ebn0_db"])
        passes = {"config2": 4, "config3": 30, "config4": 2}[name]   # bench.LEGS: timed loops of >= ~0.3 s
        assert lg["steps"] == passes * P and lg["value"] > 0 and lg["ms_per_launch"] > 0
        assert abs(lg["value"] - b / (lg["ms_per_step"] / 1e3)) <= 1e-6 * lg["value"]
        for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "launch_ms"):
            assert k in lg["roofline"], (name, k)
        assert "clock" in lg
    # config [4]'s bytes are served beyond L2 mostly by the Infinity Cache: labelled so, HBM fraction beside it
    r4 = legs["config4"]["roofline"]
    assert r4["bound"].startswith("memory-side") and r4["peak"] == 8600.0 and 0 < r4["hbm_frac"]
    # the engine clock over the timed loop (amdsmi gpu_metrics), or the reason it could not be read
    clk = d["clock"]
    assert "clock_mhz" in clk or "error" in clk, clk
    if "clock_mhz" in clk:
        assert 500 < clk["clock_mhz"] <= 2500 and clk["samples"] >= 1
        # an on-chip bound (a counter record of this exact configuration: the full-size run) also carries its
        # fraction at the clock the loop ran at (peaks scale with the clock)
        r = d["roofline"]
        if r["bound"] in ("lds", "valu"):
            assert r["clock_mhz"] == clk["clock_mhz"]
            assert abs(r["frac_at_clock"] - r["frac"] * 2400.0 / clk["clock_mhz"]) < 1e-9
    assert d["ranks"]["per_rank"][0]["clock"] == clk
