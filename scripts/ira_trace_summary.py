"""Summarise scripts/ira_trace.sh kernel traces: per IRA kernel the mean duration, and per stream (queue) the idle gap
between one IRA kernel's end and the next one's start, over the last decode of each trace.
    python scripts/ira_trace_summary.py gpurun_out/kt/base_st1 ..."""
import csv
import gzip
import glob
import sys
from collections import defaultdict


def rows(d):
    f = glob.glob(f"{d}/**/*kernel_trace.csv*", recursive=True)[0]
    op = gzip.open if f.endswith(".gz") else open
    with op(f, "rt") as fh:
        return list(csv.DictReader(fh))


def short(name):
    for k in ("k_ira_vn", "k_ira_cn", "k_ira_load", "k_ira_out", "fillBuffer"):
        if k in name:
            return k
    return None


for d in sys.argv[1:]:
    rs = [r for r in rows(d) if short(r["Kernel_Name"])]
    rs.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the last decode: from the last k_ira_load group (chunks of one decode follow each other; take the final third)
    loads = [i for i, r in enumerate(rs) if short(r["Kernel_Name"]) == "k_ira_load"]
    nch = len(loads) // 3  # warmup + 2 timed decodes per trace
    first = loads[-nch] if nch else 0
    sel = rs[first:]
    t0 = int(sel[0]["Start_Timestamp"]); t1 = max(int(r["End_Timestamp"]) for r in sel)
    dur = defaultdict(list)
    byq = defaultdict(list)
    for r in sel:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        dur[short(r["Kernel_Name"])].append(e - s)
        byq[r.get("Queue_Id") or r.get("Stream_Id")].append((s, e))
    gaps = []
    for q, iv in byq.items():
        iv.sort()
        gaps += [b[0] - a[1] for a, b in zip(iv, iv[1:])]
    busy = 0; cur_s = cur_e = None  # union of kernel intervals (any queue)
    for s, e in sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in sel):
        if cur_e is None or s > cur_e:
            if cur_e is not None: busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    print(f"{d}: chunks {nch}, decode span {(t1 - t0) / 1e6:.2f} ms, kernels busy (union) {busy / 1e6:.2f} ms, "
          f"queues {len(byq)}")
    for k, v in sorted(dur.items()):
        print(f"   {k:12s} n={len(v):5d} mean {sum(v) / len(v) / 1e3:7.2f} us  total {sum(v) / 1e6:7.2f} ms")
    gaps.sort()
    if gaps:
        print(f"   same-queue gaps: n={len(gaps)} mean {sum(gaps) / len(gaps) / 1e3:.2f} us, median "
              f"{gaps[len(gaps) // 2] / 1e3:.2f} us, total {sum(gaps) / 1e6:.2f} ms")
