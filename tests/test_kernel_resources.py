"""Every kernel a BASELINE.json configuration dispatches is spill-free: no VGPR spills and no scratch, read
from the gfx950 code objects' AMDGPU metadata notes of the built libldpc_hip.so (no GPU needed;
scripts/kernel_resources.py).  SGPR spills go to VGPR lanes (v_writelane), not to memory, and are allowed.
Config [2]'s resident kernel is checked on the disassembly as well: no scratch anywhere (round 4 kept five values
set before its iteration loop and read after it in scratch — 63 MB of stores per launch; its epilogue now
recomputes them, the lane id by v_mbcnt).  The tanh-SP register kernels come in two passes (qc.hip / qc_sl_sp.h PASS): the plain
loop (PASS 1) every input without an exact-zero LLR runs, checked here, and the a == 1 rule's loop (PASS 2) for the
waves / units whose LLRs hold an exact zero (erasures, quantized LLRs), which may spill: it runs only there.

    [1] (648,1/2) min-sum 50 it          k_qc_ms_ph<Wifi648_12, false, false, 0>
    [2] (1944,5/6) tanh-SP, 16-QAM OFDM   k_qc_sp_rs<Wifi1944_56, 1> (fixed count), k_qc_sp_sl<Wifi1944_56, *, 1>
                                          (early stop; the fixed-count sliced kernel remains for QC_SL_SP_RS=0)
    [3] (1296,2/3) 5-bit min-sum 20 it ES k_qc_qms_pk<Wifi1296_23, *, *>  (packed fp16, two codewords per lane)
    [4] DVB-S2 64800 rate 1/2, 50 it      IRA kernels (ira.hip: k_ira_vn<8, *>, k_ira_cn<8, true, *>, k_ira_load,
                                          k_ira_out); the generic CSR kernels at degree bound 8 (k_vn_ms/k_cn_ms,
                                          k_vn_sp/k_cn_sp, k_load_llr, k_final) for any other H and for tanh-SP
    drop-in decode_bits on (648,1/2)      k_qc_sp_st<Wifi648_12, false, 1>
"""
import os
import re
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

BASELINE_KERNELS = [
    r"k_qc_ms_ph<ldpc::Wifi648_12, false, false, 0>",
    r"k_qc_sp_sl<ldpc::Wifi1944_56, (true|false), 1>",
    r"k_qc_qms_pk<ldpc::Wifi1296_23, (true|false), (true|false)>",
    r"k_vn_ms<8, (true|false), \d>",
    r"k_cn_ms<8, (true|false), \d>",
    r"k_vn_sp<float, 8, false, \d>",
    r"k_cn_sp<float, 8, false, \d>",
    r"k_load_llr<float>",
    r"k_final<float, 32, (true|false)>",
    r"k_qc_sp_st<ldpc::Wifi648_12, false, 1>",
    r"k_ira_vn<(8|16), (true|false)>",
    r"k_ira_cn<(8|24), true, (true|false)>",
    r"k_ira_load\(",
    r"k_ira_out\(",
]
MAX_SPILL_OUTSIDE_LOOP = {r"k_qc_sp_rs<ldpc::Wifi1944_56, 1>": 0}
MAX_SCRATCH_IN_LOOP = 0


@pytest.fixture(scope="module")
def resources():
    import kernel_resources as kr
    if not os.path.exists(kr.READELF) or not shutil.which("c++filt"):
        pytest.skip("llvm-readelf / c++filt not available")
    if not os.path.exists(kr.DEFAULT_LIB):
        pytest.fail("libldpc_hip.so is not built")
    ks = kr.kernels()
    names = sorted(ks)
    return {d: ks[n] for n, d in zip(names, kr.demangle(names))}


@pytest.mark.parametrize("pattern", BASELINE_KERNELS)
def test_baseline_config_kernels_do_not_spill(resources, pattern):
    hits = {d: r for d, r in resources.items() if re.search(r"ldpc::" + pattern, d)}
    assert hits, f"no kernel matches {pattern}"
    for d, r in hits.items():
        assert r.get("vgpr_spill_count", 0) == 0, (d, r)
        assert r.get("private_segment_fixed_size", 0) == 0, (d, r)


@pytest.mark.parametrize("pattern", sorted(MAX_SPILL_OUTSIDE_LOOP))
def test_resident_kernel_spills_only_outside_the_iteration_loop(resources, pattern):
    """At most the listed number of spilled VGPRs, and at most a handful of scratch instructions in the kernel's
    iteration loop (its longest backward branch, scripts/isa_mix.py), none in its phases: the loop runs from
    registers and LDS."""
    import kernel_resources as kr
    from isa_mix import kernel_lines, main_loop
    hits = {d: r for d, r in resources.items() if re.search(r"ldpc::" + pattern, d)}
    assert len(hits) == 1, hits
    (d, r), = hits.items()
    assert r.get("vgpr_spill_count", 0) <= MAX_SPILL_OUTSIDE_LOOP[pattern], (d, r)
    _, lines = kernel_lines(kr.DEFAULT_LIB, "k_qc_sp_rsINS_11Wifi1944_56ELi1E")
    loop = main_loop(lines)
    assert len(loop) > 1000, len(loop)
    scratch = [op for _, op, _, _ in loop if op.startswith("scratch_")]
    assert len(scratch) <= MAX_SCRATCH_IN_LOOP, scratch


GENERIC_KERNELS = r"ldpc::k_(vn_sp|vn_spw|cn_sp|vn_ms|cn_ms|final|load_llr)<"


def test_generic_kernels_use_no_scratch(resources):
    """The generic CSR kernels (any H: the path for codes without QC tables, weights, initial messages and
    fp64) at every degree bound and vector width keep their per-slot arrays in registers: their slot loops
    are compile-time (static_for), so no instantiation falls back to private memory (the V = 2, MAXD 12/16
    tanh-SP kernels did with #pragma unroll: (1296,2/3) generic tanh-SP 0.85 -> 1.33 M cw/s)."""
    hits = {d: r for d, r in resources.items() if re.search(GENERIC_KERNELS, d)}
    assert len(hits) > 40, sorted(hits)
    bad = {d: r for d, r in hits.items() if r.get("vgpr_spill_count", 0) or r.get("private_segment_fixed_size", 0)}
    assert not bad, bad


def _kernel_bodies():
    """{mangled kernel symbol: [instructions]} over every gfx950 code object of the built library."""
    import subprocess
    import kernel_resources as kr
    objdump = os.path.join(os.path.dirname(kr.READELF), "llvm-objdump")
    out = {}
    for k, co in enumerate(kr.code_objects(kr.DEFAULT_LIB)):
        path = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"ldpc_co_{os.getpid()}_{k}.co")
        with open(path, "wb") as f:
            f.write(co)
        dis = subprocess.run([objdump, "-d", path], capture_output=True, text=True, check=True).stdout
        os.unlink(path)
        for m in re.finditer(r"\n[0-9a-f]+ <(_Z[^>]+)>:\n(.*?)(?=\n[0-9a-f]+ <_Z|\Z)", dis, re.S):
            out[m.group(1)] = [l.split("//")[0].strip() for l in m.group(2).splitlines() if l.startswith("\t")]
    return out


def test_lds_row_rotation_kernels_write_m0_once():
    """Every kernel that rotates lanes through an LDS row (ds_write_addtid_b32 stores to M0 + 4 * lane: the
    headline k_qc_ms_ph in every non-early-stop instantiation — plain, alpha / beta / both normalised, float-
    register quantized — and any other variant built with its LDS-row option) sets M0 once, in inline asm
    before the loop: the compiler must not write M0 anywhere else in it (nor read it for another purpose), or
    the rotations would store to the wrong row."""
    bodies = _kernel_bodies()
    rot = {k: v for k, v in bodies.items() if any("ds_write_addtid_b32" in i for i in v)}
    ph = [k for k in bodies if k.startswith("_ZN4ldpc10k_qc_ms_ph") and "ELb0ELb0E" in k]  # QUANT=0, EARLY=0
    assert len(ph) == 4 and set(ph) <= set(rot), (sorted(ph), sorted(rot))      # NORM 0..3 all rotate via LDS rows
    for k, insts in rot.items():
        m0 = [i for i in insts if re.search(r"\bm0\b", i)]
        assert len(m0) == 1 and m0[0].startswith("s_mov_b32 m0,"), (k, m0)
    head = "_ZN4ldpc10k_qc_ms_phINS_10Wifi648_12ELb0ELb0ELi0EEEvPKfliffffffiPhPfPi"
    assert sum("ds_write_addtid_b32" in i for i in rot[head]) >= 88, "LDS-row rotations missing"


def test_no_sign_extended_64bit_salu_literals():
    """64-bit SALU moves of a 32-bit literal with bit 31 set: the gfx950 SALU zero-extends the literal, so such a
    move is only right when the intended value is the zero extension.  The one legitimate use in the library is
    0xffffffff (a ballot's low half, 0x00000000ffffffff); any other (the compiler lowering a sign-extended
    64-bit lane mask that way — it decoded garbage in every Z = 54 kernel) fails here.  qc_common.h sel_lanes
    passes such masks complemented."""
    pat = re.compile(r"^\s*s_\w+_b64\s+[^/]*?(0x[89a-fA-F][0-9a-fA-F]{7})\b")
    bad = {}
    for k, insts in _kernel_bodies().items():
        hits = [i for i in insts if (m := pat.match(i)) and m.group(1).lower() != "0xffffffff"]
        if hits:
            bad[k] = hits[:3]
    assert not bad, bad
