"""A fixed slice of the randomised parity sweep (scripts/parity_stress.py) as a regression test: the
first 160 trials of seed 101 — random code, algorithm, parameters, iteration count, batch, Eb/N0, erasures, LLR
scale, fixed count or early stop, device or host inputs, fp64 — every kernel path against its checker, no
mismatch (the ulp-level a == 1 case of DESIGN §3.5 is the sweep's documented allowance)."""
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
