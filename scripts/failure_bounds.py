#!/usr/bin/env python3
"""Re-measure tests/softparity.py FAILURE_BOUNDS after a change of the fp32 arithmetic: read the JSON-line records
the soft-parity checks log (LDPC_PARITY_LOG, run with LDPC_PARITY_MEASURE=1 so only rule (i) is asserted) and
print the table — per (kind, golden set, implementation) the largest count of failure entries where the
reference's fp32 meets 1e-5 and ours does not, and the largest maximum on failures rounded up in the third digit.

    LDPC_PARITY_MEASURE=1 LDPC_PARITY_LOG=/tmp/o.jsonl python -m pytest tests/test_oracle_golden.py -m "not gpu"
    LDPC_PARITY_MEASURE=1 LDPC_PARITY_LOG=gpurun_out/g.jsonl python -m pytest tests -m gpu   (on the GPU box)
    python scripts/failure_bounds.py /tmp/o.jsonl gpurun_out/g.jsonl
"""
import json
import math
import sys

COUNT = {"z": "failures_entries_rel_gt_1e-5_where_ref_f32_within", "p1": "failures_entries_gt_tol_where_ref_f32_within"}
MAX = {"z": "max_rel_on_failures", "p1": "max_abs_on_failures"}


def key(rec):
    parts = rec["label"].split()
    if parts[0] == "oracle-ds":
        return rec["kind"], " ".join(parts[1:3]), "oracle"
    return rec["kind"], " ".join(parts[:2]), "gpu"


def up3(x):
    if x <= 0:
        return 0.0
    e = math.floor(math.log10(x)) - 2
    return math.ceil(x / 10.0**e) * 10.0**e


def main():
    table = {}
    for path in sys.argv[1:]:
        for line in open(path):
            rec = json.loads(line)
            if rec.get("kind") not in COUNT or COUNT[rec["kind"]] not in rec:
                continue
            k = key(rec)
            c, m = rec[COUNT[rec["kind"]]], rec[MAX[rec["kind"]]]
            oc, om = table.get(k, (0, 0.0))
            table[k] = (max(oc, c), max(om, m))
    for k in sorted(table, key=lambda k: (k[2] != "gpu", k[1], k[0] != "z")):
        c, m = table[k]
        if c:
            print(f'    ("{k[0]}", "{k[1]}", "{k[2]}"): ({c}, {up3(m):.2e}),')


if __name__ == "__main__":
    main()
