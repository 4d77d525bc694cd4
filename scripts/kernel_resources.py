#!/usr/bin/env python3
"""Per-kernel register / spill / scratch figures of a built library, read from the gfx950 code objects'
AMDGPU metadata notes (no GPU needed).

    python scripts/kernel_resources.py [LIB.so] [--filter SUBSTR]

libldpc_hip.so's .hip_fatbin section holds one clang offload bundle per compiled source; each bundle's
gfx950 entry is an ELF code object whose NT_AMDGPU_METADATA note lists, per kernel, .vgpr_count,
.vgpr_spill_count, .sgpr_spill_count and .private_segment_fixed_size (llvm-readelf --notes prints it).
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_LIB = os.path.join(ROOT, "ldpc-sims_amd", "ldpc_amd", "libldpc_hip.so")
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(lib):
    """Yield the gfx950 code objects (bytes) of every offload bundle in the library."""
    data = open(lib, "rb").read()
    i = data.find(MAGIC)
    while i >= 0:
        n = struct.unpack_from("<Q", data, i + 24)[0]
        off = i + 32
        for _ in range(n):
            o, sz, tl = struct.unpack_from("<QQQ", data, off)
            off += 24
            triple = data[off:off + tl].decode()
            off += tl
            if "gfx950" in triple and sz:
                yield data[i + o:i + o + sz]
        i = data.find(MAGIC, i + 24)


def kernels(lib=DEFAULT_LIB):
    """{kernel symbol: {vgpr_count, vgpr_spill_count, sgpr_spill_count, private_segment_fixed_size, ...}}"""
    out = {}
    for co in code_objects(lib):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            txt = subprocess.run([READELF, "--notes", f.name], capture_output=True, text=True, check=True).stdout
        # one "- .args: ..." block per kernel; the fields below appear once per block
        for blk in re.split(r"\n\s+- \.agpr_count:", txt)[1:]:
            rec = {}
            for key in ("name", "symbol", "vgpr_count", "vgpr_spill_count", "sgpr_spill_count",
                        "private_segment_fixed_size", "sgpr_count"):
                m = re.search(r"\n\s+\." + key + r":\s+(\S+)", blk)
                if m:
                    v = m.group(1)
                    rec[key] = int(v) if v.isdigit() else v
            if "name" in rec:
                out[rec["name"]] = rec
    return out


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.splitlines() if r.returncode == 0 else list(names)


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    lib = args[0] if args else DEFAULT_LIB
    flt = next((a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--filter=")), "")
    ks = kernels(lib)
    names = sorted(k for k in ks if flt in k)
    for n, d in zip(names, demangle(names)):
        r = ks[n]
        print(f"vgpr {r.get('vgpr_count', '?'):>4} spill {r.get('vgpr_spill_count', '?'):>4} "
              f"sgpr_spill {r.get('sgpr_spill_count', '?'):>3} scratch {r.get('private_segment_fixed_size', '?'):>5}  {d}")
