#!/usr/bin/env python3
"""Static instruction mix of a kernel's main loop in a built library (no GPU): disassemble the gfx950 code
objects (scripts/kernel_resources.py's bundle walk), find the kernel whose symbol contains SUBSTR, take the
longest backward branch's body (the iteration loop) and count its instructions by class — VALU,
transcendental VALU (quarter rate), LDS, waitcnt, nop (hazard wait states), SALU, barriers.

    python scripts/isa_mix.py LIB.so SUBSTR [--top N] [--phases]
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_resources import code_objects  # noqa: E402

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def classify(op):
    if op.startswith(("v_exp", "v_log", "v_rcp", "v_sqrt", "v_rsq", "v_sin", "v_cos")):
        return "valu_trans"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith("s_"):
        return "salu"
    return op


def kernel_lines(lib, sub):
    """[(offset from the kernel start, opcode, operands, branch target offset or None)]"""
    for co in code_objects(lib):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            out = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", f.name], capture_output=True, text=True).stdout
        m = re.search(r"^([0-9a-f]+) <(\w*%s\w*)>:" % re.escape(sub), out, re.M)
        if not m:
            continue
        base = int(m.group(1), 16)
        lines = []
        for ln in out[m.end():].splitlines():
            if re.match(r"^[0-9a-f]+ <", ln):
                break
            mm = re.match(r"\s*(\S+)(.*?)//\s*([0-9A-Fa-f]+):(.*)$", ln)
            if not mm:
                continue
            t = re.search(r"<[^>]*\+0x([0-9a-f]+)>", mm.group(4))
            lines.append((int(mm.group(3), 16) - base, mm.group(1), mm.group(2).strip(),
                          int(t.group(1), 16) if t and mm.group(1).startswith("s_") and "branch" in mm.group(1) else None))
        return m.group(2), lines
    raise SystemExit(f"no kernel matching {sub}")


def main_loop(lines):
    best = None
    for a, op, _, t in lines:
        if t is not None and t < a and (best is None or a - t > best[1] - best[0]):
            best = (t, a)
    return [x for x in lines if best[0] <= x[0] <= best[1]] if best else lines


def mix(ins):
    c = collections.Counter(classify(op) for _, op, _, _ in ins)
    nops = 0
    for _, op, rest, _ in ins:
        if op == "s_nop":
            n = re.match(r"(\d+)", rest)
            nops += (int(n.group(1)) if n else 0) + 1
    return dict(c), nops


def main():
    lib, sub = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 0
    name, lines = kernel_lines(lib, sub)
    loop = main_loop(lines)
    c, nops = mix(loop)
    print(name[:100])
    print("  loop instructions:", len(loop), c, "nop wait states:", nops)
    if top:
        print("  ", collections.Counter(op for _, op, _, _ in loop).most_common(top))
    if "--phases" in sys.argv:  # the loop split at its s_barrier instructions
        bars = [i for i, (_, op, _, _) in enumerate(loop) if op == "s_barrier"] + [len(loop)]
        lo = 0
        for b in bars:
            if b > lo:
                print("   phase", mix(loop[lo:b]))
            lo = b


if __name__ == "__main__":
    main()
