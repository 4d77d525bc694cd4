"""The C-ABI library loads and exports every symbol include/ldpc_abi.h declares (no GPU needed)."""
import ctypes
import os
import re

import numpy as np

from conftest import ROOT
from ldpc_amd import _abi


def _declared():
    src = open(os.path.join(ROOT, "include", "ldpc_abi.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ldpc_[a-z_0-9]+)\s*\(", src)))


def test_header_and_binding_agree():
    assert sorted(_abi.EXPORTS) == _declared()


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_abi.LIB_PATH)
    for name in _declared():
        assert hasattr(lib, name), name


def test_no_torch_types_in_header():
    src = open(os.path.join(ROOT, "include", "ldpc_abi.h")).read()
    assert "torch" not in src.split("*/", 1)[1].lower() or "at::" not in src
    assert "hipStream_t" not in re.sub(r"/\*.*?\*/", "", src, flags=re.S)


def test_argument_validation_without_gpu():
    lib = _abi.load()
    assert lib.ldpc_version().startswith(b"ldpc-mi355x")
    g = ctypes.c_void_p()
    rc = lib.ldpc_graph_create(0, 4, 0, None, None, 0, ctypes.byref(g))
    assert rc == _abi.LDPC_EINVAL and b"bad graph" in lib.ldpc_last_error()
    rp = np.array([0, 2, 1], np.int32)  # non-monotone
    ci = np.array([0, 1], np.int32)
    rc = lib.ldpc_graph_create(2, 2, 2, rp.ctypes.data, ci.ctypes.data, 0, ctypes.byref(g))
    assert rc == _abi.LDPC_EINVAL
    rp = np.array([0, 2], np.int32)
    ci = np.array([1, 0], np.int32)  # not ascending
    rc = lib.ldpc_graph_create(1, 2, 2, rp.ctypes.data, ci.ctypes.data, 0, ctypes.byref(g))
    assert rc == _abi.LDPC_EINVAL and b"ascending" in lib.ldpc_last_error()
    sh = np.array([[0, 30]], np.int32)  # shift >= z
    rc = lib.ldpc_graph_create_qc(1, 2, 27, sh.ctypes.data, 0, ctypes.byref(g))
    assert rc == _abi.LDPC_EINVAL
    assert lib.ldpc_graph_destroy(None) == 0
    assert lib.ldpc_device_count() >= 0


def test_abi_revision_matches_header_and_binding():
    """ldpc_decode's signature changed in round 5 (iters_used before the stream): the library reports the
    header's LDPC_ABI_VERSION and the binding refuses any other revision."""
    src = open(os.path.join(ROOT, "include", "ldpc_abi.h")).read()
    hdr = int(re.search(r"#define LDPC_ABI_VERSION (\d+)", src).group(1))
    lib = _abi.load()
    assert lib.ldpc_abi_version() == hdr == _abi.ABI_VERSION == 2


def test_loader_refuses_other_abi_revision(tmp_path):
    import subprocess
    so = tmp_path / "libold.so"
    c = tmp_path / "old.c"
    c.write_text("int ldpc_abi_version(void) { return 1; }\n")
    subprocess.check_call(["gcc", "-shared", "-fPIC", "-o", str(so), str(c)])
    import pytest
    with pytest.raises(ImportError, match="ABI revision 1"):
        _abi.load(str(so))


def test_params_struct_layout():
    assert ctypes.sizeof(_abi.Params) == 36
