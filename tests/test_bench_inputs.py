"""Every file bench.py reads on the GPU box must travel there: gpurun snapshots the repo minus the
patterns in .gpurunignore (tar --exclude semantics), so a default input path that one of them matches
would make bench silently lose that input (the reference-CPU record sat under ./profiles/r02)."""
import argparse
import fnmatch
import os
import sys

from conftest import ROOT


def _patterns():
    out = []
    for line in open(os.path.join(ROOT, ".gpurunignore")):
        line = line.strip()
        if line and not line.startswith("#"):
            out.append(line)
    return out


def excluded(relpath, patterns):
    """tar --exclude: './x' anchors at the top; a bare pattern matches any trailing run of path components
    (so 'name' or '*.log' at any depth); excluding a directory excludes everything below it."""
    parts = relpath.split("/")
    for p in patterns:
        for k in range(1, len(parts) + 1):
            prefix = "/".join(parts[:k])
            if p.startswith("./"):
                if fnmatch.fnmatchcase(prefix, p[2:]):
                    return p
            else:
                for i in range(k):
                    if fnmatch.fnmatchcase("/".join(parts[i:k]), p):
                        return p
    return None


def _bench_defaults():
    sys.path.insert(0, ROOT)
    import bench
    src = open(bench.__file__).read()
    # the default input paths bench.py declares (argparse defaults under ROOT)
    paths = []
    for key in ("--ref-cpu-json", "--counters-json"):
        i = src.index(f'"{key}"')
        seg = src[i:src.index("\n", src.index("help=", i))]
        expr = seg[seg.index("default=") + len("default="):seg.index(",\n") if ",\n" in seg else None]
        paths.append(eval(expr.split(",\n")[0].rstrip(","), {"os": os, "ROOT": ROOT}))
    return paths


def test_matcher_semantics():
    pats = ["./profiles/r02", "*.log", "SURVEY.md"]
    assert excluded("profiles/r02/ref_cpu_wifi648.json", pats) == "./profiles/r02"
    assert excluded("profiles/ref_cpu_wifi648.json", pats) is None
    assert excluded("a/b/x.log", pats) == "*.log"
    assert excluded("docs/SURVEY.md", pats) == "SURVEY.md"
    assert excluded("bench.py", pats) is None


def test_bench_inputs_travel_to_the_gpu_box():
    pats = _patterns()
    paths = _bench_defaults()
    assert len(paths) == 2
    for p in paths:
        rel = os.path.relpath(p, ROOT)
        assert os.path.exists(p), f"bench input {rel} missing"
        assert excluded(rel, pats) is None, f"bench input {rel} is excluded by .gpurunignore ({excluded(rel, pats)})"


def test_gpu_run_sources_travel():
    """Sources, built libraries and fixtures the GPU tests / smoke / bench load are not excluded either."""
    pats = _patterns()
    keep = ["bench.py", "__graft_entry__.py", "ldpc-sims_amd/ldpc_amd/libldpc_hip.so", "oracle/liboracle.so",
            "oracle/oracle.py", "tests/golden/bp_wifi648_12_sp_it50.npz", "profiles/counters.json"]
    for rel in keep:
        assert excluded(rel, pats) is None, rel
