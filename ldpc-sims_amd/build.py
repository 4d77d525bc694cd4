"""Build libldpc_hip.so in-tree for gfx950 (hipcc cross-compiles; no GPU needed).

Each source compiles to its own object (in parallel), then one link; per-file flags below.
"""
import os
import re
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
# (source, object, extra flags): generic_run.hip is compiled once per driver instantiation of the generic
# decoder (precision x algorithm x early stop) so its kernel templates build in parallel units.
_RUNS = [("sp32", "float", 0, 0), ("sp32_es", "float", 0, 1), ("sp64", "double", 0, 0), ("sp64_es", "double", 0, 1),
         ("ms32", "float", 1, 0), ("ms32_es", "float", 1, 1)]
SRCS = [("abi.hip", "abi.hip.o", []), ("generic.hip", "generic.hip.o", [])] + [
    ("generic_run.hip", f"generic_run_{n}.o", [f"-DRUN_T={t}", f"-DRUN_MS={ms}", f"-DRUN_ES={es}", f"-DRUN_NAME=generic_run_{n}"])
    for (n, t, ms, es) in _RUNS] + [("qc.hip", "qc.hip.o", []), ("qc_sl.hip", "qc_sl.hip.o", []), ("qc_pk.hip", "qc_pk.hip.o", []),
           ("qc_sl_es.hip", "qc_sl_es.hip.o", []), ("qc_es.hip", "qc_es.hip.o", []),
           ("channel.hip", "channel.hip.o", []), ("ira.hip", "ira.hip.o", [])]
OUT = os.path.join(HERE, "ldpc_amd", "libldpc_hip.so")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
         "-ffp-contract=off",  # min-sum must round exactly like oracle/ldpc_oracle.c (no FMA contraction)
         "-fno-slp-vectorize",  # v_pk_* f32 pairs need aligned register pairs: +100 VGPRs in the QC kernel
         "-Wall", "-Wno-unused-function"]
# The QC register kernels compute on finite values only (min/max of |messages|, no NaN can arise from
# finite LLRs): with no-NaN semantics hipcc drops the canonicalising v_max before each v_min and the
# min(+inf, x) of the first slot: -6 % instructions in an instruction-fetch-bound loop.  Results for
# finite inputs are identical.  (-mno-amdgpu-ieee would also do it, but a kernel whose IEEE-mode
# attribute differs from the device library's cannot inline any library routine, blockDim included.)
# iterative-ilp scheduling: +2 % on the (648,1/2) stored min-sum loop (A/B, 34.4 -> 35.1 M cw/s), same code
# otherwise (the loop is latency- and issue-limited at the 128-VGPR / 4-waves budget).
SCHED = ["-mllvm", "--amdgpu-sched-strategy=iterative-ilp"]
PER_FILE = {"qc.hip": ["-fno-honor-nans", *SCHED], "qc_sl.hip": ["-fno-honor-nans", *SCHED],
            "qc_pk.hip": ["-fno-honor-nans"], "qc_sl_es.hip": ["-fno-honor-nans"], "qc_es.hip": ["-fno-honor-nans"]}  # iterative-ilp crashes the register allocator on qc_pk (ROCm 7.2)


def _hip_includes(src):
    """The csrc/*.hip files `src` #includes (one level: the per-variant translation units)."""
    with open(src) as f:
        names = re.findall(r'^\s*#\s*include\s+"([^"]+\.hip)"', f.read(), re.M)
    return [os.path.join(os.path.dirname(src), n) for n in names]


def build(force: bool = False, verbose: bool = False, out: str = OUT, defines=(), per_file=True, qc_flags=None) -> str:
    srcs = [os.path.join(HERE, "csrc", s) for (s, _, _) in SRCS]
    deps = srcs + [os.path.join(HERE, "csrc", "common.h"), os.path.join(ROOT, "include", "ldpc_abi.h")]
    deps += [os.path.join(HERE, "csrc", f) for f in os.listdir(os.path.join(HERE, "csrc")) if f.endswith(".h")]
    deps.append(os.path.abspath(__file__))
    if not force and os.path.exists(out) and os.path.getmtime(out) >= max(os.path.getmtime(d) for d in deps):
        return out
    if qc_flags is not None:
        PER_FILE["qc.hip"] = qc_flags
    objdir = os.path.join(os.path.dirname(os.path.abspath(out)), "." + os.path.basename(out) + ".objs")
    os.makedirs(objdir, exist_ok=True)
    common = ["hipcc", *[f for f in FLAGS if f != "-shared"], *[f"-D{d}" for d in defines],
              "-I", os.path.join(ROOT, "include"), "-I", os.path.join(HERE, "csrc")]
    objs, cmds = [], []
    hdrs = [d for d in deps if d.endswith(".h")] + [os.path.abspath(__file__)]
    for (name, oname, extra) in SRCS:
        src = os.path.join(HERE, "csrc", name)
        obj = os.path.join(objdir, oname)
        objs.append(obj)
        # an object is reused when newer than its source, the .hip files it includes (qc_es.hip is qc.hip
        # built again with other flags), every header and this script (same flags)
        if (not force and not defines and os.path.exists(out) and os.path.exists(obj)
                and os.path.getmtime(obj) >= max(os.path.getmtime(d) for d in [src, *_hip_includes(src), *hdrs])):
            continue
        cmds.append([*common, *extra, *(PER_FILE.get(name, []) if per_file else []), "-c", "-o", obj, src])
    link = ["hipcc", "--offload-arch=gfx950", "-fPIC", "-shared", "-o", out, *objs]

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)

    with ThreadPoolExecutor(max_workers=max(1, len(cmds))) as ex:
        list(ex.map(run, cmds))
    run(link)
    return out


TEST_KERNELS = [(os.path.join(ROOT, "tests", "kern", "cn_rows.hip"), os.path.join(ROOT, "tests", "kern", "libcnrows.so"))]


def build_test_kernels(force: bool = False, verbose: bool = False) -> None:
    """The test-only kernel libraries (tests/kern/*.hip: instantiations of csrc routines the GPU tests check
    directly), same flags as the product objects."""
    hdrs = [os.path.join(HERE, "csrc", f) for f in os.listdir(os.path.join(HERE, "csrc")) if f.endswith(".h")]
    for src, out in TEST_KERNELS:
        if not force and os.path.exists(out) and os.path.getmtime(out) >= max(os.path.getmtime(d) for d in [src, *hdrs]):
            continue
        cmd = ["hipcc", *FLAGS, "-I", os.path.join(ROOT, "include"), "-I", os.path.join(HERE, "csrc"), "-o", out, src]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)


if __name__ == "__main__":
    # python build.py [--force] [--out PATH] [-DNAME=VAL ...]
    args = sys.argv[1:]
    out = args[args.index("--out") + 1] if "--out" in args else OUT
    defs = [a[2:] for a in args if a.startswith("-D")]
    qcf = next((a.split("=", 1)[1].split() for a in args if a.startswith("--qc-flags=")), None)
    print(build(force="--force" in args or bool(defs) or "--no-per-file" in args or qcf is not None, verbose=True,
                out=out, defines=defs, per_file="--no-per-file" not in args, qc_flags=qcf))
    if out == OUT and not defs:
        build_test_kernels(force="--force" in args, verbose=True)
