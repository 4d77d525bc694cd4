import pickle

import numpy as np

from ldpc_amd.sweep import save


def test_pkl_uses_reference_schema(tmp_path):
    r = dict(snrdb=np.arange(3.0), uncoded_ber=np.ones(3) * 0.1, coded_ber=np.ones(3) * 0.01,
             coded_bler=np.ones(3) * 0.2, codewords=np.array([5, 5, 5]), seconds=1.0, config={})
    p = tmp_path / "r.pkl"
    save(r, str(p))
    with open(p, "rb") as f:   # our own file
        d = pickle.load(f)
    assert set(d) == {"snrdb", "uncoded_ber", "coded_ber", "coded_bler"}   # evaluate_quantized.py:156-160
    assert all(isinstance(v, np.ndarray) for v in d.values())
    save(r, str(tmp_path / "r.json"))
