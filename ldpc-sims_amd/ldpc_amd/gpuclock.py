"""Engine clock and power of the decode GPU around a timed region (bench.py's `clock` record).

The headline kernel is power-limited (2.15–2.23 GHz traced where the other kernels run at
2.38–2.40), so a throughput number means little without the clock it ran at.  A background thread polls
amdsmi's gpu_metrics table (firmware-updated, ~1 ms) while the timed loop runs: `current_gfxclks` (one
engine clock per XCD), `current_socket_power`, and the firmware's PPT (package power limit) residency
counter.  Measurement plumbing only: nothing here touches the decode, and every failure (no amdsmi, no
permission, a field the firmware does not fill) becomes an "error" entry instead of an exception.
"""
from __future__ import annotations

import threading
import time

_NA = (None, "N/A")
_INIT = []  # amdsmi initialised once per process (the library is process-global)


def _num(x):
    return None if x in _NA or isinstance(x, str) else x


def _handle_for(device_index: int):
    """The amdsmi processor handle of torch's device `device_index` (matched by PCI domain:bus; amdsmi may
    list every GPU of the host while HIP sees only the ones this process was given)."""
    import amdsmi
    import torch
    props = torch.cuda.get_device_properties(device_index)
    want = (getattr(props, "pci_domain_id", None), getattr(props, "pci_bus_id", None))
    handles = amdsmi.amdsmi_get_processor_handles()
    if not handles:
        raise RuntimeError("amdsmi lists no GPU")
    for h in handles:
        bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)  # "dddd:bb:dd.f"
        dom, bus = bdf.split(":")[:2]
        if want[1] is not None and (int(dom, 16), int(bus, 16)) == (want[0] or 0, want[1]):
            return h, bdf
    if len(handles) == 1:
        return handles[0], amdsmi.amdsmi_get_gpu_device_bdf(handles[0])
    raise RuntimeError(f"no amdsmi GPU at PCI {want} among {len(handles)}")


class ClockSampler:
    """`with ClockSampler(dev) as cs: <timed loop>` then `cs.summary()`."""

    def __init__(self, device_index: int, period_s: float = 0.002):
        self.period = period_s
        self.samples = []      # (t, mean gfxclk MHz over XCDs, min over XCDs, socket W)
        self.err = None
        self._acc0 = self._acc1 = None
        self._stop = threading.Event()
        self._thr = None
        try:
            import amdsmi
            if not _INIT:
                amdsmi.amdsmi_init()
                _INIT.append(True)
            self._amdsmi = amdsmi
            self.h, self.bdf = _handle_for(device_index)
        except Exception as e:  # no amdsmi / no permission / no match: record why, measure nothing
            self.err = f"{type(e).__name__}: {e}"

    def _read(self):
        m = self._amdsmi.amdsmi_get_gpu_metrics_info(self.h)
        clks = [c for c in (_num(x) for x in (m.get("current_gfxclks") or [])) if c]
        if not clks and _num(m.get("current_gfxclk")):
            clks = [m["current_gfxclk"]]
        return m, clks

    # the firmware's throttle residency counters: per accumulation tick, whether the package sat at that limit
    LIMITS = ("ppt", "socket_thm", "vr_thm", "hbm_thm", "prochot")

    def _acc(self, m):
        return (_num(m.get("accumulation_counter")),) + tuple(_num(m.get(f"{k}_residency_acc")) for k in self.LIMITS)

    def _run(self):
        while not self._stop.is_set():
            try:
                m, clks = self._read()
                if clks:
                    self.samples.append((time.perf_counter(), sum(clks) / len(clks), min(clks),
                                         _num(m.get("current_socket_power"))))
            except Exception as e:
                self.err = f"{type(e).__name__}: {e}"
                return
            self._stop.wait(self.period)

    def __enter__(self):
        if self.err is None:
            try:
                self._acc0 = self._acc(self._read()[0])
            except Exception as e:
                self.err = f"{type(e).__name__}: {e}"
                return self
            self._thr = threading.Thread(target=self._run, daemon=True)
            self._thr.start()
        return self

    def __exit__(self, *exc):
        if self._thr is not None:
            self._stop.set()
            self._thr.join()
            try:
                self._acc1 = self._acc(self._read()[0])
            except Exception:
                pass
        return False

    def summary(self, since=None) -> dict:
        """`since`: a time.perf_counter() value; samples taken before it (a warmup's tail) are left out."""
        if self.err is not None and not self.samples:
            return {"error": self.err, "source": "amdsmi gpu_metrics"}
        s = self.samples if since is None else [x for x in self.samples if x[0] >= since]
        out = {"source": "amdsmi gpu_metrics: current_gfxclks (mean over XCDs), current_socket_power, "
                         "throttle residency accumulators; polled every %.0f ms over the timed loop" % (self.period * 1e3),
               "pci": self.bdf, "samples": len(s)}
        if s:
            mean = [x[1] for x in s]
            out.update(clock_mhz=sum(mean) / len(mean), clock_mhz_min=min(x[2] for x in s),
                       clock_mhz_max=max(mean))
            pw = [x[3] for x in s if x[3] is not None]
            if pw:
                out["socket_power_w"] = sum(pw) / len(pw)
        a0, a1 = self._acc0, self._acc1
        if a0 and a1 and None not in (a0[0], a1[0]) and a1[0] > a0[0]:
            ticks = a1[0] - a0[0]
            lim = {k: (a1[i + 1] - a0[i + 1]) / ticks for i, k in enumerate(self.LIMITS)
                   if a0[i + 1] is not None and a1[i + 1] is not None}
            if "ppt" in lim:
                out["ppt_limited_frac"] = lim["ppt"]   # the package at its power limit
            if lim:
                out["limit_residency"] = lim           # every throttle limit's share of the loop
            # amdsmi's averaged power reading lags the load: over windows of tens of ms it under-reads
            out["note"] = "power and residency are firmware averages; meaningful over windows of >= ~0.3 s"
        if self.err is not None:
            out["error"] = self.err
        return out
