"""A fixed slice of the randomised parity sweep (scripts/parity_stress.py) as a regression test: the
first 160 trials of seed 101 — random code, algorithm, parameters, iteration count, batch, Eb/N0, erasures, LLR
scale, fixed count or early stop, device or host inputs, fp64 — every kernel path against its checker, no
mismatch.  fp32 tanh-SP is held to its specification (the oracle's (D, S) form: bits, 1e-5 z and iteration counts on
the codewords the oracle decodes, exact zeros of the a == 1 rule) and bit for bit to the generic kernels, with no
allowance (round 6: the rule is per codeword in every kernel)."""
import importlib.util
import os

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_parity_sweep_slice(tmp_path):
    pytest.importorskip("torch")
    spec = importlib.util.spec_from_file_location("parity_stress", os.path.join(ROOT, "scripts", "parity_stress.py"))
    ps = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ps)
    rc = ps.main(["--trials", "160", "--seconds", "600", "--seed", "101", "--extended", "--out", str(tmp_path)])
    assert rc == 0, open(tmp_path / "summary.json").read()
