"""Per-dispatch means of scripts/ira_pmc.sh counters for the IRA variable / check kernels, per library variant.
    python scripts/ira_pmc_summary.py gpurun_out/ipmc base s8"""
import csv
import glob
import sys
from collections import defaultdict

root, names = sys.argv[1], sys.argv[2:]


def load(name):
    acc = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per-dispatch values]
    for f in sorted(glob.glob(f"{root}/{name}_p*/**/*counter_collection.csv", recursive=True)):
        per = defaultdict(float)
        kern = {}
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r["Kernel_Name"]
                key = ("k_ira_vn" if "k_ira_vn" in k else "k_ira_cn" if "k_ira_cn" in k else None)
                if key is None:
                    continue
                per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
                kern[r["Dispatch_Id"]] = key
        for (d, c), v in per.items():
            acc[kern[d]][c].append(v)
    return acc


data = {n: load(n) for n in names}
for kern in ("k_ira_vn", "k_ira_cn"):
    print(kern)
    cs = sorted(set().union(*(data[n][kern].keys() for n in names)))
    for c in cs:
        vals = []
        for n in names:
            v = data[n][kern].get(c)
            vals.append(f"{sum(v) / len(v):14.4g}" if v else f"{'-':>14s}")
        g = data[names[0]][kern].get("GRBM_GUI_ACTIVE")
        print(f"  {c:40s}" + "".join(vals))
