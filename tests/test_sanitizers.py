"""CPU sanitizer builds (SURVEY.md §5 "race detection / sanitizers").

* The CPU oracle (oracle/ldpc_oracle.c) under AddressSanitizer + UndefinedBehaviorSanitizer, driven by
  oracle/sanitize_main.c over every entry point on random and degenerate graphs (empty checks, unconnected
  variables, degree-1 checks, no edges, long rows).  This build catches an out-of-range edge access like the
  one the (D, S) form's first version had for an empty check.
* The host side of the drop-in (ldpc-sims_amd/csrc/host_pipeline.h: the persistent HostPool workers, the
  two-slot staging pipeline ldpc_decode_bits_host runs) under ThreadSanitizer, and under ASan + UBSan, against
  a fake asynchronous copy engine (tests/host/test_host_pipeline.cpp): ragged chunks, 1-16 threads, error
  injection at every submit, two concurrent callers.

GPU-side sanitizers (ASan on gfx950 needs xnack) are not available on the GPU pool; these are host-only.
"""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

CSRC = os.path.join(ROOT, "ldpc-sims_amd", "csrc")


def _build_and_run(tmp_path, compiler, srcs, flags, name, env_extra=None, libs=()):
    exe = str(tmp_path / name)
    cmd = [compiler, *flags, "-o", exe, *srcs, *libs]
    b = subprocess.run(cmd, capture_output=True, text=True)
    if b.returncode != 0 and "sanitize" in b.stderr and ("unrecognized" in b.stderr or "cannot find" in b.stderr):
        pytest.skip(f"{compiler} lacks the sanitizer runtime: {b.stderr[-300:]}")
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ, OMP_NUM_THREADS="4", **(env_extra or {}))
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
    return r


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_oracle_asan_ubsan(tmp_path):
    _build_and_run(tmp_path, "gcc", [os.path.join(ROOT, "oracle", "ldpc_oracle.c"), os.path.join(ROOT, "oracle", "sanitize_main.c")],
                   ["-std=c11", "-O1", "-g", "-fopenmp", "-ffp-contract=off", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all"], "oracle_san", libs=["-lm"])


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_host_pipeline_tsan(tmp_path):
    _build_and_run(tmp_path, "g++", [os.path.join(ROOT, "tests", "host", "test_host_pipeline.cpp")],
                   ["-std=c++17", "-O1", "-g", "-pthread", "-fsanitize=thread", "-I", CSRC], "pipe_tsan",
                   env_extra={"TSAN_OPTIONS": "halt_on_error=1"})


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_host_pipeline_asan_ubsan(tmp_path):
    _build_and_run(tmp_path, "g++", [os.path.join(ROOT, "tests", "host", "test_host_pipeline.cpp")],
                   ["-std=c++17", "-O1", "-g", "-pthread", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-I", CSRC], "pipe_asan")
