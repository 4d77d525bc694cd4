import pickle

import numpy as np

from ldpc_amd.sweep import PKL_KEYS, save

# the keys plots.py:12-27 reads unconditionally (written at evaluate_quantized.py:155-172)
PLOTS_READS = ("snrdb", "uncoded_ber", "coded_ber", "coded_bler", "uncoded_ber_nn", "coded_ber_nn", "coded_bler_nn",
               "uncoded_ber_quantized", "coded_ber_quantized", "coded_bler_quantized", "wmse_nn", "wmse_quantized")


def _result(npts=3, adc=False):
    r = dict(snrdb=np.arange(float(npts)), uncoded_ber=np.ones(npts) * 0.1, coded_ber=np.ones(npts) * 0.01,
             coded_bler=np.ones(npts) * 0.2, codewords=np.array([5] * npts), seconds=1.0, config={})
    if adc:
        r.update(uncoded_ber_quantized=np.ones(npts) * 0.2, coded_ber_quantized=np.ones(npts) * 0.02,
                 coded_bler_quantized=np.ones(npts) * 0.3, wmse_quantized=np.ones(npts) * 0.5)
    return r


def test_pkl_has_every_key_plots_reads(tmp_path):
    for adc in (False, True):
        p = tmp_path / f"r{adc}.pkl"
        save(_result(4, adc), str(p))
        with open(p, "rb") as f:   # our own file
            d = pickle.load(f)
        assert set(PLOTS_READS) <= set(d) and set(d) == set(PKL_KEYS)
        for k in PLOTS_READS:
            assert isinstance(d[k], np.ndarray) and d[k].shape == (4,) and d[k].dtype == np.float64, k
        assert np.isnan(d["coded_ber_nn"]).all() and np.isnan(d["wmse_nn"]).all()   # NN: out of scope
        assert np.isnan(d["coded_ber_quantized"]).all() != adc
        assert np.array_equal(d["coded_ber"], np.ones(4) * 0.01)
    save(_result(), str(tmp_path / "r.json"))


def test_checkpoint_key_digests():
    """The sweep checkpoint key's identities: H's digest depends on H's nonzeros and shape, not on
    its container; the library digest is the sha1 of the loaded file."""
    import hashlib
    from ldpc_amd import _abi
    from ldpc_amd.codes import get_code
    from ldpc_amd.sweep import code_digest
    H = get_code("peg64_32")[0]
    assert code_digest(H) == code_digest(H.astype(np.int64)) == code_digest(H.copy())
    assert code_digest(H) != code_digest(H[::-1].copy())
    H3 = H.copy()
    H3[0, np.flatnonzero(H3[0] == 0)[0]] = 1                 # one more edge
    assert code_digest(H3) != code_digest(H)
    dv = get_code("dvbs2_12")[0]                               # SparseCode container
    assert len(code_digest(dv)) == 40
    with open(_abi.load()._ldpc_path, "rb") as f:
        assert _abi.library_digest() == hashlib.sha1(f.read()).hexdigest()
