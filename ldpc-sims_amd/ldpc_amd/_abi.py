"""ctypes binding of libldpc_hip.so (include/ldpc_abi.h).

There is deliberately no fallback: if the HIP library is missing, importing ldpc_amd raises.  The
decoder exists only as the gfx950 code in ``ldpc-sims_amd/csrc``.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_NAME = "libldpc_hip.so"
LIB_PATH = os.path.join(HERE, LIB_NAME)

LDPC_OK, LDPC_EINVAL, LDPC_EHIP, LDPC_ENOMEM, LDPC_EUNSUPPORTED = 0, -1, -2, -3, -4
ALGO_TANH_SP, ALGO_MIN_SUM, ALGO_QMIN_SUM = 0, 1, 2
F_EARLY_STOP, F_DEVICE_PTRS, F_F64, F_SOFT_Z, F_FORCE_GENERIC = 1, 2, 4, 8, 16

# every symbol include/ldpc_abi.h declares (tests/test_abi.py checks the header and the .so agree)
EXPORTS = (
    "ldpc_graph_create", "ldpc_graph_create_qc", "ldpc_graph_destroy", "ldpc_graph_info",
    "ldpc_workspace_size", "ldpc_decode_ex", "ldpc_decode", "ldpc_count_errors", "ldpc_awgn_llr",
    "ldpc_random_bits", "ldpc_ofdm_tx", "ldpc_ofdm_demod", "ldpc_adc_quantize", "ldpc_weights_layout",
    "ldpc_decode_weighted", "ldpc_decode_x0", "ldpc_decode_bits_host", "ldpc_last_error", "ldpc_device_count",
    "ldpc_version", "ldpc_kernel_path", "ldpc_abi_version",
)
ABI_VERSION = 2  # LDPC_ABI_VERSION of include/ldpc_abi.h this binding is written for


class LdpcError(RuntimeError):
    """Raised for a non-zero return code; carries ldpc_last_error()."""

    def __init__(self, code, msg):
        super().__init__(f"ldpc error {code}: {msg}")
        self.code = code


class Params(ctypes.Structure):
    _fields_ = [("iters", ctypes.c_int32), ("algo", ctypes.c_int32), ("flags", ctypes.c_int32),
                ("clamp", ctypes.c_float), ("alpha", ctypes.c_float), ("beta", ctypes.c_float),
                ("qmax", ctypes.c_int32), ("app_max", ctypes.c_int32), ("qstep", ctypes.c_float)]


class BPWeights(ctypes.Structure):
    """ldpc_bp_weights: device pointers (vn, llr, fin, fin_llr), NULL = all ones."""
    _fields_ = [("vn", ctypes.c_void_p), ("llr", ctypes.c_void_p), ("fin", ctypes.c_void_p),
                ("fin_llr", ctypes.c_void_p)]


_lib = None


def load(path: str | None = None):
    global _lib
    if _lib is not None and path is None:
        return _lib
    # LDPC_LIB: alternative build of the same library (used to A/B kernel variants in one GPU session)
    p = path or os.environ.get("LDPC_LIB") or LIB_PATH
    try:
        # torch ships its own libamdhip64.so (soname libamdhip64.so.7).  Loading torch first makes our
        # DT_NEEDED libamdhip64.so.7 resolve to that same runtime instead of a second copy from /opt/rocm
        # (two HIP runtimes in one process see different device sets).
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(p):
        raise ImportError(f"{p} not found: the HIP decoder is not built (run `python __graft_entry__.py`); "
                          "there is no CPU fallback")
    L = ctypes.CDLL(p)
    try:
        got = ctypes.CFUNCTYPE(ctypes.c_int)(("ldpc_abi_version", L))()
    except AttributeError:
        got = 1  # revision 1 libraries predate the symbol
    if got != ABI_VERSION:
        raise ImportError(f"{p}: ABI revision {got}, this binding needs {ABI_VERSION} (include/ldpc_abi.h "
                          "LDPC_ABI_VERSION); rebuild the library")
    vp, i32, i64, sz = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t
    gpp = ctypes.POINTER(ctypes.c_void_p)
    L.ldpc_graph_create.argtypes = [i32, i32, i32, vp, vp, i32, gpp]
    L.ldpc_graph_create_qc.argtypes = [i32, i32, i32, vp, i32, gpp]
    L.ldpc_graph_destroy.argtypes = [vp]
    L.ldpc_graph_info.argtypes = [vp, vp, vp, vp, vp]
    L.ldpc_workspace_size.argtypes = [vp, i64, ctypes.POINTER(Params), ctypes.POINTER(sz)]
    L.ldpc_decode_ex.argtypes = [vp, vp, i64, ctypes.POINTER(Params), vp, vp, vp, vp, sz, vp]
    L.ldpc_decode.argtypes = [vp, vp, i64, i32, ctypes.c_float, i32, i32, vp, vp, vp, vp]
    L.ldpc_count_errors.argtypes = [vp, vp, i64, i32, i32, vp, vp]
    L.ldpc_awgn_llr.argtypes = [vp, vp, i64, i32, ctypes.c_float, ctypes.c_uint64, i64, vp]
    L.ldpc_random_bits.argtypes = [vp, i64, i32, ctypes.c_uint64, i64, vp]
    L.ldpc_ofdm_tx.argtypes = [vp, i64, i32, i32, ctypes.c_float, ctypes.c_uint64, i64, vp, vp, vp]
    L.ldpc_ofdm_demod.argtypes = [vp, i64, i32, i32, ctypes.c_float, vp, vp, vp]
    L.ldpc_adc_quantize.argtypes = [vp, i64, i32, ctypes.c_double, ctypes.c_double, vp, vp, vp]
    L.ldpc_weights_layout.argtypes = [vp, ctypes.POINTER(i64), ctypes.POINTER(i64)]
    L.ldpc_decode_weighted.argtypes = [vp, vp, i64, ctypes.POINTER(Params), ctypes.POINTER(BPWeights), vp, vp, vp,
                                       vp, sz, vp]
    L.ldpc_decode_x0.argtypes = [vp, vp, i64, ctypes.POINTER(Params), ctypes.POINTER(BPWeights), vp, vp, vp, vp,
                                 vp, sz, vp]
    L.ldpc_decode_bits_host.argtypes = [vp, vp, i64, ctypes.POINTER(Params), vp, i64, i32]
    for f in ("ldpc_graph_create", "ldpc_graph_create_qc", "ldpc_graph_destroy", "ldpc_graph_info",
              "ldpc_workspace_size", "ldpc_decode_ex", "ldpc_decode", "ldpc_count_errors", "ldpc_awgn_llr",
              "ldpc_random_bits", "ldpc_ofdm_tx", "ldpc_ofdm_demod", "ldpc_adc_quantize", "ldpc_weights_layout", "ldpc_decode_weighted",
              "ldpc_decode_x0", "ldpc_decode_bits_host", "ldpc_device_count", "ldpc_abi_version"):
        getattr(L, f).restype = ctypes.c_int
    L.ldpc_last_error.restype = ctypes.c_char_p
    L.ldpc_version.restype = ctypes.c_char_p
    L.ldpc_kernel_path.argtypes = [vp, ctypes.POINTER(Params)]
    L.ldpc_kernel_path.restype = ctypes.c_char_p
    L._ldpc_path = p
    if path is None:
        _lib = L
    return L


_digests: dict = {}


def library_digest(path: str | None = None) -> str:
    """sha1 of the library file in use (the build identity: every kernel change rebuilds it)."""
    import hashlib
    p = path or load()._ldpc_path
    if p not in _digests:
        h = hashlib.sha1()
        with open(p, "rb") as f:
            for blk in iter(lambda: f.read(1 << 20), b""):
                h.update(blk)
        _digests[p] = h.hexdigest()
    return _digests[p]


def check(rc: int):
    if rc != LDPC_OK:
        raise LdpcError(rc, load().ldpc_last_error().decode(errors="replace"))
    return rc
