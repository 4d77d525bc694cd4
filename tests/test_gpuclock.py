"""ldpc_amd.gpuclock's summary (no GPU): clock mean / min / max over the samples, socket power, and each
throttle limit's residency share from the firmware's accumulators over the loop — `ppt_limited_frac` kept
for the power limit, missing counters left out rather than guessed."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ldpc-sims_amd"))

from ldpc_amd.gpuclock import ClockSampler  # noqa: E402


def _sampler(samples, m0, m1, err=None):
    c = ClockSampler.__new__(ClockSampler)
    c.err, c.samples, c.period, c.bdf = err, samples, 0.002, "0000:00:00.0"
    c._acc0, c._acc1 = (c._acc(m0), c._acc(m1)) if m0 is not None else (None, None)
    return c


def test_summary_clock_power_and_limits():
    m0 = {"accumulation_counter": 100, "ppt_residency_acc": 10, "socket_thm_residency_acc": 0,
          "vr_thm_residency_acc": 5, "hbm_thm_residency_acc": 0, "prochot_residency_acc": "N/A"}
    m1 = {"accumulation_counter": 300, "ppt_residency_acc": 60, "socket_thm_residency_acc": 0,
          "vr_thm_residency_acc": 105, "hbm_thm_residency_acc": 0, "prochot_residency_acc": "N/A"}
    s = _sampler([(0.0, 2100.0, 2050, 900.0), (0.002, 2200.0, 2150, 1000.0)], m0, m1).summary()
    assert s["clock_mhz"] == 2150.0 and s["clock_mhz_min"] == 2050 and s["clock_mhz_max"] == 2200.0
    assert s["socket_power_w"] == 950.0 and s["samples"] == 2
    assert s["ppt_limited_frac"] == 0.25
    assert s["limit_residency"] == {"ppt": 0.25, "socket_thm": 0.0, "vr_thm": 0.5, "hbm_thm": 0.0}


def test_summary_without_accumulators_or_amdsmi():
    s = _sampler([(0.0, 2000.0, 2000, None)], None, None).summary()
    assert s["clock_mhz"] == 2000.0 and "socket_power_w" not in s and "limit_residency" not in s
    e = _sampler([], None, None, err="ModuleNotFoundError: amdsmi").summary()
    assert e["error"].startswith("ModuleNotFoundError") and "clock_mhz" not in e
