"""The committed counter records are what scripts/counters_summary.py derives from the committed raw rocprofv3
CSVs (profiles/r05/prof/): every record in profiles/counters.json is recomputable, uses the timed loop's launches
(one per Eb/N0 point) and implies a clock within the 2.4 GHz peak (plus the per-dispatch allowance of a multi-launch
decode); and the summary rejects a record whose counted launches are not the traced ones (implied clock above the
peak)."""
import csv
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

SUMMARY = os.path.join(ROOT, "scripts", "counters_summary.py")
PROF = os.path.join(ROOT, "profiles", "r05", "prof")
SEL = {"c1_wifi648_minsum50": ["--kernel", "k_qc_ms_ph", "--last", "11"],
       "c1_wifi648_tanh50": ["--kernel", "k_qc_sp_st", "--last", "11"],
       "c2_wifi1944_tanh50_16qam": ["--kernel", "k_qc_sp_rs", "--last", "11"],
       "c3_wifi1296_q5_20es": ["--kernel", "k_qc_qms_pk", "--last", "11"],
       "c4_dvbs2_minsum50": ["--decode-kernels", "k_ira_load,k_ira_vn,k_ira_cn,k_ira_out", "--chunks", "21",
                             "--last", "1"]}


def _records():
    return {r["name"]: r for r in json.load(open(os.path.join(ROOT, "profiles", "counters.json")))}


def test_every_baseline_config_has_a_record():
    recs = _records()
    assert sorted(recs) == sorted(SEL)
    for r in recs.values():
        per = r["derived"].get("dispatches_per_decode")
        allow = 1.03 + (per * 8e-3 / r["kernel_stats"]["mean_ms"] if per else 0.0)
        assert r["derived"]["clock_ghz"] <= 2.4 * allow
        assert r["kernel_stats"]["calls"] == int(SEL[r["name"]][-1])      # one launch per Eb/N0 point
        # the traced mean and bench's event-timed launch agree (the same launches were counted and timed)
        assert abs(r["kernel_stats"]["mean_ms"] / r["bench"]["launch_ms_events"] - 1) < 0.03


@pytest.mark.parametrize("name", sorted(SEL))
def test_record_recomputes_from_raw_csvs(name):
    d = os.path.join(PROF, f"prof_{name}")
    if not os.path.isdir(d):
        pytest.skip("raw profiles not in this checkout")
    out = subprocess.run([sys.executable, SUMMARY, d, "--name", name, *SEL[name]], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    assert json.loads(out.stdout) == _records()[name]


def test_rejects_counts_from_other_launches(tmp_path):
    """A record whose cycles over the traced duration imply more than the peak clock is refused."""
    d = tmp_path / "prof_fake"
    (d / "ks").mkdir(parents=True)
    (d / "pmc1").mkdir()
    json.dump({"config": {"code": "x"}, "value": 1.0, "ms_per_step": 1.0, "roofline": {"launch_ms": 1.0}},
              open(d / "bench.json", "w"))
    with open(d / "ks" / "run_kernel_trace.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Dispatch_Id", "Start_Timestamp", "End_Timestamp"])
        for i in range(3):
            w.writerow(["k_test(int)", i, 0, 1_000_000])                 # 1 ms each
    with open(d / "pmc1" / "run_counter_collection.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Dispatch_Id", "Counter_Name", "Counter_Value"])
        for i in range(3):
            w.writerow(["k_test(int)", i, "GRBM_GUI_ACTIVE", 8 * 3.0e6])  # 3e6 cycles per XCD in 1 ms: 3 GHz
            w.writerow(["k_test(int)", i, "SQ_INSTS_VALU", 1.0e6])
    out = subprocess.run([sys.executable, SUMMARY, str(d), "--name", "fake", "--kernel", "k_test", "--last", "3"],
                         capture_output=True, text=True)
    assert out.returncode != 0 and "REJECTED" in (out.stderr + out.stdout)


def test_chunked_decodes(tmp_path):
    """--chunks K: a decode whose first kernel is launched once per chunk (the IRA path) is K dispatches of it;
    the per-decode sums and the decode count follow, and a count that is not whole decodes is refused."""
    d = tmp_path / "prof_chunks"
    (d / "ks").mkdir(parents=True)
    (d / "pmc1").mkdir()
    json.dump({"config": {"code": "x"}, "value": 1.0, "ms_per_step": 1.0, "roofline": {"launch_ms": 0.3}},
              open(d / "bench.json", "w"))
    rows, i = [], 0
    for dec in range(4):                       # 4 decodes x 3 chunks x (load, vn) dispatches
        for ch in range(3):
            for k in ("k_load(int)", "k_vn(int)"):
                rows.append((k, i))
                i += 1
    with open(d / "ks" / "run_kernel_trace.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Dispatch_Id", "Start_Timestamp", "End_Timestamp"])
        for k, j in rows:
            w.writerow([k, j, 0, 50_000])           # 0.05 ms each: 0.3 ms per decode
    with open(d / "pmc1" / "run_counter_collection.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Dispatch_Id", "Counter_Name", "Counter_Value"])
        for k, j in rows:
            w.writerow([k, j, "GRBM_GUI_ACTIVE", 8 * 1.0e5])   # 1e5 cycles per dispatch per XCD: 2 GHz
            w.writerow([k, j, "SQ_INSTS_VALU", 10.0])
    args = [sys.executable, SUMMARY, str(d), "--name", "c", "--decode-kernels", "k_load,k_vn", "--last", "2"]
    out = subprocess.run(args + ["--chunks", "3"], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    r = json.loads(out.stdout)
    assert r["kernel_stats"]["calls"] == 2 and abs(r["kernel_stats"]["mean_ms"] - 0.3) < 1e-9
    assert abs(r["counters_per_launch"]["SQ_INSTS_VALU"] - 60.0) < 1e-9 and abs(r["derived"]["clock_ghz"] - 2.0) < 1e-9
    bad = subprocess.run(args + ["--chunks", "5"], capture_output=True, text=True)
    assert bad.returncode != 0 and "whole decodes" in (bad.stderr + bad.stdout)
