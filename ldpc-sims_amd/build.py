"""Build libldpc_hip.so in-tree for gfx950 (hipcc cross-compiles; no GPU needed)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRCS = ["abi.hip", "generic.hip", "qc.hip", "channel.hip"]
OUT = os.path.join(HERE, "ldpc_amd", "libldpc_hip.so")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
         "-ffp-contract=off",  # min-sum must round exactly like oracle/ldpc_oracle.c (no FMA contraction)
         "-fno-slp-vectorize",  # v_pk_* f32 pairs need aligned register pairs: +100 VGPRs in the QC kernel
         "-Wall", "-Wno-unused-function"]


def build(force: bool = False, verbose: bool = False, out: str = OUT, defines=()) -> str:
    srcs = [os.path.join(HERE, "csrc", s) for s in SRCS]
    deps = srcs + [os.path.join(HERE, "csrc", "common.h"), os.path.join(ROOT, "include", "ldpc_abi.h")]
    deps += [os.path.join(HERE, "csrc", f) for f in os.listdir(os.path.join(HERE, "csrc")) if f.endswith(".h")]
    deps.append(os.path.abspath(__file__))
    if not force and os.path.exists(out) and os.path.getmtime(out) >= max(os.path.getmtime(d) for d in deps):
        return out
    cmd = ["hipcc", *FLAGS, *[f"-D{d}" for d in defines], "-I", os.path.join(ROOT, "include"),
           "-I", os.path.join(HERE, "csrc"), "-o", out, *srcs]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    return out


if __name__ == "__main__":
    # python build.py [--force] [--out PATH] [-DNAME=VAL ...]
    args = sys.argv[1:]
    out = args[args.index("--out") + 1] if "--out" in args else OUT
    defs = [a[2:] for a in args if a.startswith("-D")]
    print(build(force="--force" in args or bool(defs), verbose=True, out=out, defines=defs))
