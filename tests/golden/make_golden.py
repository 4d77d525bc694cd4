#!/usr/bin/env python3
"""Generate the golden vectors under tests/golden/ by running the REFERENCE decoder itself.

Run in the build container only (needs /root/reference; never on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What it records (all .npz, numeric arrays only — loadable with allow_pickle=False):
  * peg64_32.npz           H and G exported from ``bp/parity.py:7-44``.
  * bp_peg64_*.npz         For Eb/N0 {0,2,4} dB x (iters, clamp) in {(3,20),(5,10),(10,10),(10,100),(50,10)}:
                           the input llr (float32, log P1/P0 convention), the reference's fp32 output
                           ``p1 = BeliefPropagation(H, iters)(0, llr, clamp)`` (``bp/bp.py:43-51``), the same
                           module run in float64 (``.double()``), and ``np.round(p1)`` hard bits.
  * bp_peg64_trace.npz     Per-iteration c2v messages ``x`` (check-order, ``bp/bp.py:46-47``) for 16 codewords,
                           5 iterations, clamp 10 — pins edge ordering and the c2v update itself.
  * decode_bits_peg64.npz  ``decode_bits(llrs, H, 5, 48, 10)`` (``ofdm/ofdm_functions.py:131-163``) with N=100,
                           so rows 96..99 (N % batch_size) exercise the "remainder rows stay 0" quirk.
  * bp_wifi648.npz         802.11n (648,1/2) H (ldpc_amd.codes) through the reference BP: 16 codewords,
                           iters 5, clamp 10, Eb/N0 1 and 2 dB, fp32 and fp64.
  * demod_ofdm.npz         ``demodulate_signal`` (``ofdm_functions.py:63-78``) on a fixed received vector:
                           pins the reference's LLR formula/sign convention for the channel front end.
  * adc_quantizer.npz      ``quantizer`` (``:37-51``) at fixed clips (incl. the lo > hi corner) and
                           ``gen_qdata`` (``:118-128``, AGC clip = std * ratio) on a complex64-valued stream.
  * bp_x0.npz              the forward with non-zero initial messages x (bp/bp.py:43-47).
  * bp_weighted_peg64.npz  weighted BP: the reference module with random per-layer ``input_weight`` /
                           ``llr_weight`` set in memory (``bp_vc.py:19,24``), 5 iterations, fp32 and fp64.
  * bp_<code>_sp.npz       802.11n (648,1/2), (1296,2/3), (1944,5/6): p1 and z, 5 iterations, clamp 10.
  * bp_<code>_sp_it<k>.npz the same at 50 / 20 / 10 iterations (one reference layer looped, checked bitwise
                           against BeliefPropagation(H, 5) first).
  * bp_wifi1944_56_sp_it50_cl20.npz  BASELINE config [2]: (1944,5/6) 50 iterations, clamp 20, 16-QAM OFDM LLRs
                           from the on-device front end (c2_16qam_llrs.npz, scripts/gen_c2_llrs_gpu.py): fp32,
                           .double() and the f32-bound .double() (wifi1944c2).
  * e2e_wifi648_qpsk_ofdm.npz  the reference's whole receiver chain (bits, encode_bits, modulate_bits, gen_data's
                           32-point OFDM over AWGN, demodulate_signal) into decode_bits(llrs, H, 50, 40, 10) on
                           the (648,1/2) code, 96 rows per Es/N0 point (rows 80..95 stay 0) (e2e648).
  * e2e_quantized.npz      the reference's quantized chain (3-bit ADC via gen_qdata, evaluate_quantized.py) into
                           decode_bits at clamp 20: (64,32) at 3 iterations, (648,1/2) at 50; LLRs with exact
                           zeros (e2eq).
  * bp_zeros.npz           clustered exact-zero LLRs (2-3 zeros in a third of the checks, both signs): (64,32) and
                           (648,1/2), 1/2/3/5 iterations, clamp 10 and 20, p1 and z, fp32 and .double() (zeros).
  * bp_wifi648_12_sp_it50_cl20.npz  (648,1/2) 50 iterations at clamp 20, above the p-clamp ceiling; plus
                           (wificlampb32) the reference's .double() module with the fp32 module's p-clamp bound
                           swapped in at run time (f32_pclamp): p1_f64b32_* / z_f64b32_*.

    python tests/golden/make_golden.py [bp] [adc] [weighted] [wifi] [x0] [wifilong] [wificlamp] [wificlampb32] [wifi1944c2] [e2e648] [e2eq] [zeros]
"""
import contextlib
import os
import sys

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True
REF = "/root/reference/pytorch"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REF)
sys.path.insert(0, os.path.join(ROOT, "ldpc-sims_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

np.complex = complex  # the reference uses np.complex/np.float (removed in numpy 2); in-process shim only
np.float = float

from bp.bp import BeliefPropagation  # noqa: E402
from bp import parity  # noqa: E402
from ofdm import ofdm_functions as OF  # noqa: E402

from ldpc_amd.codes import wifi_code, Encoder  # noqa: E402

torch.set_num_threads(8)


def bpsk_awgn_llr(code_bits: np.ndarray, ebn0_db: float, rate: float, rng) -> np.ndarray:
    """BPSK s = 1-2c, y = s + sigma n, sigma^2 = 1/(2 R Eb/N0); LLR log P1/P0 = -2y/sigma^2."""
    sigma2 = 1.0 / (2.0 * rate * 10.0 ** (ebn0_db / 10.0))
    y = (1.0 - 2.0 * code_bits) + np.sqrt(sigma2) * rng.standard_normal(code_bits.shape)
    return (-2.0 * y / sigma2).astype(np.float32)


def run_ref(H, iters, clamp, llr32, double=False, trace=False):
    model = BeliefPropagation(H, iters)
    model.eval()
    dtype = torch.float64 if double else torch.float32
    if double:
        model = model.double()
    llr = torch.tensor(llr32, dtype=dtype)
    x = torch.zeros(llr.shape[0], model.layer_size(), dtype=dtype)
    snaps = []
    with torch.no_grad():
        if trace:  # re-run the forward loop exactly as bp.py:46-51 does, keeping x after each layer
            for layer in model.layers:
                x = layer([x, -llr]).clamp(-clamp, clamp)
                snaps.append(x.numpy().copy())
            p1 = -1 * model.final_layer([x, -llr]) + 1
        else:
            p1 = model(x, llr, clamp)
    return p1.numpy(), (np.stack(snaps) if trace else None)


def gen_bp():
    H = parity.H.astype(np.int64)
    G = parity.G.astype(np.int64)
    np.savez_compressed(os.path.join(HERE, "peg64_32.npz"), H=H, G=G)

    B = 128
    configs = [(3, 20), (5, 10), (10, 10), (10, 100), (50, 10)]
    for si, snr in enumerate([0.0, 2.0, 4.0]):
        rng = np.random.default_rng(1000 + si)
        info = rng.integers(0, 2, size=(B, 32))
        cw = (info @ G.T) % 2  # G = [I; P]: codeword = G @ info (ofdm_functions.encode_bits:11-15)
        llr = bpsk_awgn_llr(cw, snr, 0.5, rng)
        for iters, clamp in configs:
            p1_32, _ = run_ref(H, iters, clamp, llr)
            p1_64, _ = run_ref(H, iters, clamp, llr, double=True)
            name = f"bp_peg64_snr{int(snr)}_it{iters}_cl{clamp}.npz"
            np.savez_compressed(
                os.path.join(HERE, name), H=H, llr=llr, codeword=cw.astype(np.uint8), iters=iters,
                clamp=clamp, p1_f32=p1_32.astype(np.float32), p1_f64=p1_64,
                bits_f32=np.round(p1_32).astype(np.uint8), bits_f64=np.round(p1_64).astype(np.uint8))
            print(name, "bit errors vs codeword:", int((np.round(p1_32) != cw).sum()))

    # per-iteration c2v trace (check-order x), 16 codewords
    rng = np.random.default_rng(77)
    info = rng.integers(0, 2, size=(16, 32))
    cw = (info @ G.T) % 2
    llr = bpsk_awgn_llr(cw, 1.0, 0.5, rng)
    p1_32, tr32 = run_ref(H, 5, 10, llr, trace=True)
    p1_64, tr64 = run_ref(H, 5, 10, llr, double=True, trace=True)
    np.savez_compressed(os.path.join(HERE, "bp_peg64_trace.npz"), H=H, llr=llr, iters=5, clamp=10,
                        x_f32=tr32.astype(np.float32), x_f64=tr64, p1_f32=p1_32, p1_f64=p1_64)

    # the drop-in boundary itself, with a ragged tail (N % batch_size != 0)
    rng = np.random.default_rng(99)
    info = rng.integers(0, 2, size=(100, 32))
    cw = (info @ G.T) % 2
    llr64 = bpsk_awgn_llr(cw, 2.0, 0.5, rng).astype(np.float64)
    out = OF.decode_bits(llr64, H, 5, 48, 10)
    np.savez_compressed(os.path.join(HERE, "decode_bits_peg64.npz"), H=H, llrs=llr64, iters=5,
                        batch_size=48, clamp=10, out=out, out_dtype=str(out.dtype))

    # 802.11n (648,1/2) through the reference algorithm (the reference accepts any binary H)
    qc = wifi_code(648, "1/2")
    Hw = qc.H()
    enc = Encoder(Hw)
    recs = {}
    for snr in (1.0, 2.0):
        rng = np.random.default_rng(648 + int(snr))
        info = rng.integers(0, 2, size=(16, qc.k))
        cw = enc.encode(info)
        llr = bpsk_awgn_llr(cw.astype(np.float64), snr, 0.5, rng)
        p1_32, _ = run_ref(Hw, 5, 10, llr)
        p1_64, _ = run_ref(Hw, 5, 10, llr, double=True)
        tag = f"snr{int(snr)}"
        recs[f"llr_{tag}"] = llr
        recs[f"codeword_{tag}"] = cw
        recs[f"p1_f32_{tag}"] = p1_32.astype(np.float32)
        recs[f"p1_f64_{tag}"] = p1_64
        print("wifi648", tag, "bit errors:", int((np.round(p1_32) != cw).sum()))
    np.savez_compressed(os.path.join(HERE, "bp_wifi648.npz"), base=qc.base, Z=qc.Z, iters=5, clamp=10,
                        **recs)

    # channel front end: the reference's LLR demodulator on a fixed received vector
    rng = np.random.default_rng(5)
    rx = (rng.standard_normal(64) + 1j * rng.standard_normal(64)) * 0.8
    llrs, rsym = OF.demodulate_signal(rx.reshape(1, -1), 32, 10 ** (3.0 / 10))
    np.savez_compressed(os.path.join(HERE, "demod_ofdm.npz"), rx=rx, snr_db=3.0, ofdm_size=32,
                        llrs=llrs, rx_symbols=rsym)


def gen_adc():
    rng = np.random.default_rng(37)
    rx = ((rng.standard_normal(4096) + 1j * rng.standard_normal(4096)) * 0.7).astype(np.complex64)
    rx = rx.astype(np.complex128)  # complex64-representable values, so the fp32 device input is exact
    rec = dict(rx=rx)
    fixed = [(1, 0.3), (1, 1.0), (3, 0.8), (5, 2.0), (8, 1.5), (4, 0.45)]
    for i, (b, c) in enumerate(fixed):
        rec[f"q_fixed{i}"] = OF.quantizer(rx.reshape(1, -1), b, c).reshape(-1)
    rec["fixed"] = np.array(fixed, dtype=np.float64)
    agc = [(3, 1.0), (5, 2.0), (5, 3.0), (8, 1.5)]
    for i, (b, r) in enumerate(agc):
        q, qs, ql = OF.gen_qdata(rx.reshape(1, -1), 2.0, b, r, 32)
        rec[f"q_agc{i}"] = q.reshape(-1)
        rec[f"qsym_agc{i}"] = qs.reshape(-1)
        rec[f"qllr_agc{i}"] = ql.reshape(-1)
        rec[f"clip_agc{i}"] = np.max(np.std(rx.reshape(1, -1))) * r
    rec["agc"] = np.array(agc, dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, "adc_quantizer.npz"), snr_db=2.0, ofdm_size=32, **rec)


def gen_weighted():
    H = parity.H.astype(np.int64)
    G = parity.G.astype(np.int64)
    iters, clamp, B = 5, 10.0, 64
    rng = np.random.default_rng(4242)
    model = BeliefPropagation(H, iters)
    rec = {}
    for i, layer in enumerate(model.layers):
        vc = layer[0]
        vc.input_weight.data = vc.mask.data * torch.tensor(rng.uniform(0.5, 1.5, vc.mask.shape), dtype=torch.float)
        vc.llr_weight.data = torch.tensor(rng.uniform(0.5, 1.5, vc.llr_weight.shape), dtype=torch.float)
        rec[f"input_weight{i}"] = vc.input_weight.data.numpy().copy()
        rec[f"llr_weight{i}"] = vc.llr_weight.data.numpy().copy()
    fv = model.final_layer[0]
    fv.input_weight.data = fv.mask.data * torch.tensor(rng.uniform(0.5, 1.5, fv.mask.shape), dtype=torch.float)
    fv.llr_weight.data = torch.tensor(rng.uniform(0.5, 1.5, fv.llr_weight.shape), dtype=torch.float)
    rec["final_input_weight"] = fv.input_weight.data.numpy().copy()
    rec["final_llr_weight"] = fv.llr_weight.data.numpy().copy()
    model.eval()
    for snr in (1.0, 3.0):
        info = rng.integers(0, 2, size=(B, 32))
        cw = (info @ G.T) % 2
        llr = bpsk_awgn_llr(cw, snr, 0.5, rng)
        tag = f"snr{int(snr)}"
        with torch.no_grad():
            x = torch.zeros(B, model.layer_size())
            p32 = model(x, torch.tensor(llr), clamp).numpy()
            m64 = model.double()
            p64 = m64(x.double(), torch.tensor(llr, dtype=torch.float64), clamp).numpy()
            model.float()
        rec[f"llr_{tag}"] = llr
        rec[f"p1_f32_{tag}"] = p32.astype(np.float32)
        rec[f"p1_f64_{tag}"] = p64
        print("weighted", tag, "bit errors:", int((np.round(p32) != cw).sum()))
    np.savez_compressed(os.path.join(HERE, "bp_weighted_peg64.npz"), H=H, iters=iters, clamp=clamp, **rec)


def run_ref_z(H, iters, clamp, llr32, double=False):
    """The reference forward (bp/bp.py:43-51) with the final VC output z kept: the loop of bp.py:46-47,
    then z = final_layer[0]([x, -llr]) (bp_vc.py:16-27 with mask_v_final, llr_expander = I) and
    p1 = -sigmoid(z) + 1 exactly as final_layer + bp.py:51 compute it."""
    model = BeliefPropagation(H, iters)
    model.eval()
    dtype = torch.float64 if double else torch.float32
    if double:
        model = model.double()
    llr = torch.tensor(llr32, dtype=dtype)
    x = torch.zeros(llr.shape[0], model.layer_size(), dtype=dtype)
    with torch.no_grad():
        for layer in model.layers:
            x = layer([x, -llr]).clamp(-clamp, clamp)
        z = model.final_layer[0]([x, -llr])
        p1 = -1 * model.final_layer[1](z) + 1
    return p1.numpy(), z.numpy()


# 802.11n codes through the reference algorithm (the reference accepts any binary H): per code the Eb/N0
# points and codewords per point.  Memory: the reference's CV forms (B, E, E) temporaries, 16 x 6399^2 x 8 B
# = 5.2 GB each for (1944,5/6) in fp64.
WIFI_SP = [("wifi648_12", (1.0, 2.0), 64), ("wifi1296_23", (2.0, 3.0), 16), ("wifi1944_56", (3.0, 4.0), 16)]


def gen_wifi_sp():
    """bp_<code>_sp.npz: reference tanh-SP p1 and z (fp32 module and .double()), 5 iterations, clamp 10."""
    from ldpc_amd.codes import get_code
    iters, clamp = 5, 10.0
    for name, snrs, B in WIFI_SP:
        H, qc = get_code(name)
        H = np.asarray(H, dtype=np.int64)
        enc = Encoder(H)
        rate = enc.k / H.shape[1]
        rec = {}
        for snr in snrs:
            rng = np.random.default_rng(int(1000 * snr) + H.shape[1])
            info = rng.integers(0, 2, size=(B, enc.k))
            cw = enc.encode(info)
            llr = bpsk_awgn_llr(cw.astype(np.float64), snr, rate, rng)
            p32, z32 = run_ref_z(H, iters, clamp, llr)
            p64, z64 = run_ref_z(H, iters, clamp, llr, double=True)
            tag = f"snr{snr:g}".replace(".", "p")
            rec[f"llr_{tag}"] = llr
            rec[f"codeword_{tag}"] = cw.astype(np.uint8)
            rec[f"p1_f32_{tag}"] = p32.astype(np.float32)
            rec[f"z_f32_{tag}"] = z32.astype(np.float32)
            rec[f"p1_f64_{tag}"] = p64
            rec[f"z_f64_{tag}"] = z64
            print(name, tag, "bit errors:", int((np.round(p32) != cw).sum()),
                  "ref f32 vs f64: |dp1| max", float(np.abs(p32 - p64).max()), "|dz| max", float(np.abs(z32 - z64).max()),
                  flush=True)
        np.savez_compressed(os.path.join(HERE, f"bp_{name}_sp.npz"), base=qc.base, Z=qc.Z, iters=iters, clamp=clamp,
                            snrs=np.array(snrs), **rec)


# Reference runs at the iteration counts the drop-in and BASELINE configs use: (code, Eb/N0 points, codewords per
# point, iterations, reference chunk).  Memory: the reference's CV forms two (chunk, E, E) temporaries.
WIFI_SP_LONG = [("wifi648_12", (1.0, 2.0, 3.0), 64, 50, 32), ("wifi1296_23", (2.0, 2.5, 3.0), 32, 20, 16),
                ("wifi1944_56", (3.5, 4.0, 4.5), 16, 10, 8)]
# the callers' other clamps (evaluate_quantized.py:20 uses 20, evaluate_snr.py:20 uses 100): messages reach the
# reference's p-clamp ceiling log(16777215) = 16.6355 (bp_cv.py:44-47) instead of the caller's clamp
# (any clamp >= 16.64 gives the same bits: clamp 100 was run once and its file was byte-identical to this one's)
WIFI_SP_CLAMPS = [("wifi648_12", (2.0, 3.0), 64, 50, 32, 20.0)]


def run_ref_looped(model, iters, clamp, llr32, double=False):
    """The reference forward (bp/bp.py:43-51) with ONE reference layer applied `iters` times.

    Every layer of BeliefPropagation(H, iters) is a deep copy of the same Sequential(VC, Tanh, CV) with unit
    weights (bp.py:27-34, bp_vc.py:101-107), so looping layers[0] computes exactly bp.py:46-47 while holding
    one layer's E x E masks instead of `iters` of them.  Returns p1 and the final VC output z."""
    dtype = torch.float64 if double else torch.float32
    layer = model.layers[0]
    llr = torch.tensor(llr32, dtype=dtype)
    x = torch.zeros(llr.shape[0], model.layer_size(), dtype=dtype)
    with torch.no_grad():
        for _ in range(iters):
            x = layer([x, -llr]).clamp(-clamp, clamp)
        z = model.final_layer[0]([x, -llr])
        p1 = -1 * model.final_layer[1](z) + 1
    return p1.numpy(), z.numpy()


def gen_wifi_sp_long(specs=None, clamp_tag=False):
    """bp_<code>_sp_it<iters>.npz: reference tanh-SP p1 and z (fp32 module and .double()) at 50 / 20 / 10
    iterations, clamp 10, run by looping one reference layer (run_ref_looped), whose equality with the full
    BeliefPropagation(H, 5) forward is checked bitwise here first."""
    from ldpc_amd.codes import get_code
    clamp = 10.0
    specs = specs or [(*sp, 10.0) for sp in WIFI_SP_LONG]
    H0 = np.asarray(get_code("wifi648_12")[0], dtype=np.int64)
    rng = np.random.default_rng(5050)
    enc0 = Encoder(H0)
    llr0 = bpsk_awgn_llr(enc0.encode(rng.integers(0, 2, size=(8, enc0.k))).astype(np.float64), 1.5, 0.5, rng)
    m1 = BeliefPropagation(H0, 1)
    m1.eval()
    for dbl in (False, True):
        pa, za = run_ref_z(H0, 5, clamp, llr0, double=dbl)
        mm = m1.double() if dbl else m1.float()
        pb, zb = run_ref_looped(mm, 5, clamp, llr0, double=dbl)
        assert np.array_equal(pa, pb) and np.array_equal(za, zb), "looped layer != BeliefPropagation(H, 5)"
    print("looped reference layer == BeliefPropagation(H, 5), fp32 and fp64, bitwise", flush=True)
    for name, snrs, B, iters, chunk, clamp in specs:
        H, qc = get_code(name)
        H = np.asarray(H, dtype=np.int64)
        enc = Encoder(H)
        rate = enc.k / H.shape[1]
        model = BeliefPropagation(H, 1)
        model.eval()
        rec = {}
        for snr in snrs:
            rng = np.random.default_rng(int(1000 * snr) + 7 * H.shape[1] + iters)
            cw = enc.encode(rng.integers(0, 2, size=(B, enc.k)))
            llr = bpsk_awgn_llr(cw.astype(np.float64), snr, rate, rng)
            outs = {k: [] for k in ("p32", "z32", "p64", "z64")}
            for s in range(0, B, chunk):
                p32, z32 = run_ref_looped(model.float(), iters, clamp, llr[s:s + chunk])
                p64, z64 = run_ref_looped(model.double(), iters, clamp, llr[s:s + chunk], double=True)
                for k, v in zip(("p32", "z32", "p64", "z64"), (p32, z32, p64, z64)):
                    outs[k].append(v)
            p32, z32, p64, z64 = (np.concatenate(outs[k]) for k in ("p32", "z32", "p64", "z64"))
            tag = f"snr{snr:g}".replace(".", "p")
            rec[f"llr_{tag}"] = llr
            rec[f"codeword_{tag}"] = cw.astype(np.uint8)
            rec[f"p1_f32_{tag}"] = p32.astype(np.float32)
            rec[f"z_f32_{tag}"] = z32.astype(np.float32)
            rec[f"p1_f64_{tag}"] = p64
            rec[f"z_f64_{tag}"] = z64
            print(name, iters, tag, "bit errors:", int((np.round(p32) != cw).sum()),
                  "f32/f64 bit mismatches:", int((np.round(p32) != np.round(p64)).sum()),
                  "|dz| max", float(np.abs(z32 - z64).max()), flush=True)
        fname = f"bp_{name}_sp_it{iters}" + (f"_cl{int(clamp)}" if clamp_tag else "") + ".npz"
        np.savez_compressed(os.path.join(HERE, fname), base=qc.base, Z=qc.Z, iters=iters,
                            clamp=clamp, snrs=np.array(snrs), chunk=chunk, **rec)


@contextlib.contextmanager
def f32_pclamp():
    """The fp32 module's p-clamp bound in fp64 arithmetic: bp_cv.py:44-47 clamps p to +-(1 - epsilon), epsilon =
    .0000001, and torch rounds that Python float to the tensor's dtype — 0.99999988 in the fp32 module, 0.9999999
    in .double().  Inside this context torch.clamp called with exactly that bound on a float64 tensor uses
    float32(1 - 1e-7) instead, so the reference's OWN fp64 module computes the fp32 module's function (messages
    capped at log(16777215) = 16.6355 rather than log(19999999) = 16.8112).  Every other clamp — the caller's
    x.clamp(-clamp, clamp) of bp.py:47 is the Tensor method — is untouched.  Build container only."""
    orig = torch.clamp
    bound = 1 - .0000001                          # the expression bp_cv.py evaluates
    b32 = float(np.float32(bound))
    hits = [0]

    def clamp(t, *args, **kw):
        if torch.is_tensor(t) and t.dtype == torch.float64 and args == (-bound, bound) and not kw:
            hits[0] += 1
            return orig(t, -b32, b32)
        return orig(t, *args, **kw)
    torch.clamp = clamp
    try:
        yield hits
    finally:
        torch.clamp = orig


def gen_wifi_clamp_f32bound():
    """Adds p1_f64b32_<tag> / z_f64b32_<tag> to bp_wifi648_12_sp_it50_cl20.npz: the reference's .double() module
    run on the file's LLRs with the fp32 module's p-clamp bound (f32_pclamp) — the fp64 target of an fp32
    drop-in above the ceiling, from the reference itself (tests/softparity.py f64_target)."""
    from ldpc_amd.codes import qc_expand
    path = os.path.join(HERE, "bp_wifi648_12_sp_it50_cl20.npz")
    d = dict(np.load(path))
    H = qc_expand(d["base"], int(d["Z"])).astype(np.int64)
    iters, clamp, chunk = int(d["iters"]), float(d["clamp"]), int(d["chunk"])
    model = BeliefPropagation(H, 1)
    model.eval()
    for snr in d["snrs"]:
        tag = f"snr{snr:g}".replace(".", "p")
        llr = d[f"llr_{tag}"]
        ps, zs = [], []
        with f32_pclamp() as hits:
            for s in range(0, llr.shape[0], chunk):
                p64, z64 = run_ref_looped(model.double(), iters, clamp, llr[s:s + chunk], double=True)
                ps.append(p64)
                zs.append(z64)
        assert hits[0] == iters * len(ps), hits  # the bound was swapped in every CV layer call
        d[f"p1_f64b32_{tag}"] = np.concatenate(ps)
        d[f"z_f64b32_{tag}"] = np.concatenate(zs)
        print("f32-bound fp64", tag, "|dz| vs .double() max", float(np.abs(d[f"z_f64b32_{tag}"] - d[f"z_f64_{tag}"]).max()),
              "vs fp32 module", float(np.abs(d[f"z_f64b32_{tag}"] - d[f"z_f32_{tag}"]).max()), flush=True)
    np.savez_compressed(path, **d)


def gen_wifi1944_c2(llr_path=os.path.join(HERE, "c2_16qam_llrs.npz")):
    """bp_wifi1944_56_sp_it50_cl20.npz: BASELINE config [2] at its own settings through the reference itself —
    (1944,5/6), tanh-SP 50 iterations, clamp 20 (the config [2] leg's), on 16-QAM OFDM LLRs from the on-device
    front end (scripts/gen_c2_llrs_gpu.py -> c2_16qam_llrs.npz: 16 codewords at 6.0 / 6.5 dB, the waterfall):
    the fp32 module, .double(), and .double() with the fp32 module's p-clamp bound (f32_pclamp, the fp64 target
    above the ceiling), one reference layer looped (run_ref_looped; checked against BeliefPropagation(H, 5) in
    gen_wifi_sp_long)."""
    from ldpc_amd.codes import get_code
    src = np.load(llr_path)
    H, qc = get_code("wifi1944_56")
    H = np.asarray(H, dtype=np.int64)
    iters, clamp, chunk = 50, 20.0, 8
    model = BeliefPropagation(H, 1)
    model.eval()
    rec = {}
    for snr in src["snrs"]:
        tag = f"snr{snr:g}".replace(".", "p")
        llr = src[f"llr_{tag}"].astype(np.float32)
        cw = src[f"codeword_{tag}"]
        outs = {k: [] for k in ("p32", "z32", "p64", "z64", "pb", "zb")}
        for s in range(0, llr.shape[0], chunk):
            p32, z32 = run_ref_looped(model.float(), iters, clamp, llr[s:s + chunk])
            p64, z64 = run_ref_looped(model.double(), iters, clamp, llr[s:s + chunk], double=True)
            with f32_pclamp() as hits:
                pb, zb = run_ref_looped(model.double(), iters, clamp, llr[s:s + chunk], double=True)
            assert hits[0] == iters, hits
            for k, v in zip(("p32", "z32", "p64", "z64", "pb", "zb"), (p32, z32, p64, z64, pb, zb)):
                outs[k].append(v)
        p32, z32, p64, z64, pb, zb = (np.concatenate(outs[k]) for k in ("p32", "z32", "p64", "z64", "pb", "zb"))
        rec[f"llr_{tag}"] = llr
        rec[f"codeword_{tag}"] = cw.astype(np.uint8)
        rec[f"p1_f32_{tag}"] = p32.astype(np.float32)
        rec[f"z_f32_{tag}"] = z32.astype(np.float32)
        rec[f"p1_f64_{tag}"] = p64
        rec[f"z_f64_{tag}"] = z64
        rec[f"p1_f64b32_{tag}"] = pb
        rec[f"z_f64b32_{tag}"] = zb
        print("wifi1944_56 50 it clamp 20 16-QAM", tag, "bit errors:", int((np.round(p32) != cw).sum()),
              "codeword errors:", int((np.round(p32) != cw).any(1).sum()), "of", cw.shape[0],
              "|dz| f32 vs f32-bound f64", float(np.abs(z32 - zb).max()), flush=True)
    np.savez_compressed(os.path.join(HERE, "bp_wifi1944_56_sp_it50_cl20.npz"), base=qc.base, Z=qc.Z, iters=iters,
                        clamp=clamp, snrs=np.array(src["snrs"]), chunk=chunk, **rec)


def gen_e2e648():
    """e2e_wifi648_qpsk_ofdm.npz: the reference's whole receiver chain as its evaluate scripts run it
    (evaluate_snr.py:43,89,122): np.random bits, encode_bits with a generator of the (648,1/2) code,
    modulate_bits (QPSK), gen_data (32-point OFDM over AWGN, ofdm_functions.py:109-116) -> demodulate_signal LLRs,
    then decode_bits(llrs, H, 50, 40, 10) — 96 codewords per Es/N0 point, so rows 80..95 (N % batch_size) stay 0.
    Inputs are the reference's own float64 LLRs; outputs its float64 bits."""
    from ldpc_amd.codes import get_code
    H, qc = get_code("wifi648_12")
    H = np.asarray(H, dtype=np.int64)
    enc = Encoder(H)
    G = enc.encode(np.eye(enc.k, dtype=np.int64)).T.astype(np.int64)        # (n, k): cw = G @ bits mod 2
    assert not ((H @ G) % 2).any()
    B, iters, bs, clamp, ofdm = 96, 50, 40, 10, 32
    rec = {}
    snrs = (1.0, 1.5)  # the waterfall: decoded and failing rows both
    for snrdb in snrs:
        np.random.seed(int(100 * snrdb) + 648)
        bits = OF.create_bits(B * enc.k)
        cbits = OF.encode_bits(bits, G)
        tx = OF.modulate_bits(cbits)
        _, _, rx_llrs, _ = OF.gen_data(tx, snrdb, ofdm)
        llrs = rx_llrs.reshape((-1, H.shape[1]))
        out = OF.decode_bits(llrs, H, iters, bs, clamp)
        tag = f"snr{snrdb:g}".replace(".", "p")
        rec[f"llrs_{tag}"] = llrs
        rec[f"codeword_{tag}"] = cbits.reshape((-1, H.shape[1])).astype(np.uint8)
        rec[f"out_{tag}"] = out
        rows = (B // bs) * bs
        print("e2e648", tag, "bit errors in decoded rows:", int((out[:rows] != rec[f"codeword_{tag}"][:rows]).sum()),
              "tail zero:", not out[rows:].any(), flush=True)
    np.savez_compressed(os.path.join(HERE, "e2e_wifi648_qpsk_ofdm.npz"), base=qc.base, Z=qc.Z, iters=iters,
                        batch_size=bs, clamp=clamp, ofdm_size=ofdm, snrs=np.array(snrs), **rec)


def gen_e2e_quantized():
    """e2e_quantized.npz: the reference's quantized receiver chain (evaluate_quantized.py:42-46,98,137): bits ->
    encode_bits -> modulate_bits -> gen_data (32-point OFDM over AWGN) -> gen_qdata (ADC with AGC clip = std x
    ratio, ofdm_functions.py:118-128) -> demodulate_signal LLRs -> decode_bits(qrx_llrs, H, iters, bs, 20).  The
    LLRs contain exact zeros (s = +-0 in the first VC layer).  Two cases: the reference's own (64,32) with its
    evaluator's 3-bit ADC, clip ratio 1 and 3 iterations; (648,1/2) with a 5-bit ADC, clip ratio 2, 50 iterations."""
    from ldpc_amd.codes import get_code
    rec = {}
    cases = [("peg64", parity.H.astype(np.int64), np.asarray(parity.G, np.int64) if hasattr(parity, "G") else None,
              3, 100, 32, 2.0, 3, 1), ("wifi648", None, None, 50, 96, 40, 2.0, 5, 2)]
    for name, H, G, iters, B, bs, snrdb, qbits, clip_ratio in cases:
        if H is None:
            H = np.asarray(get_code("wifi648_12")[0], dtype=np.int64)
        if G is None or G.shape[0] != H.shape[1]:
            enc = Encoder(H)
            G = enc.encode(np.eye(enc.k, dtype=np.int64)).T.astype(np.int64)
        k = G.shape[1]
        assert not ((H @ G) % 2).any()
        np.random.seed(4242 + H.shape[1])
        bits = OF.create_bits(B * k)
        cbits = OF.encode_bits(bits, G)
        tx = OF.modulate_bits(cbits)
        rx_signal, _, _, _ = OF.gen_data(tx, snrdb, 32)
        _, _, qrx_llrs = OF.gen_qdata(rx_signal, snrdb, qbits, clip_ratio, 32)
        llrs = qrx_llrs.reshape((-1, H.shape[1]))
        out = OF.decode_bits(llrs, H, iters, bs, 20)
        rec[f"H_{name}"] = H.astype(np.uint8)
        rec[f"llrs_{name}"] = llrs
        rec[f"codeword_{name}"] = cbits.reshape((-1, H.shape[1])).astype(np.uint8)
        rec[f"out_{name}"] = out
        rec[f"cfg_{name}"] = np.array([iters, bs, 20, qbits, clip_ratio])
        rows = (B // bs) * bs
        print("e2eq", name, "zero LLRs:", int((llrs == 0).sum()), "distinct:", len(np.unique(llrs)),
              "bit errors in decoded rows:", int((out[:rows] != rec[f"codeword_{name}"][:rows]).sum()), flush=True)
    np.savez_compressed(os.path.join(HERE, "e2e_quantized.npz"), **rec)


def gen_x0():
    """bp_x0.npz: the reference forward with NON-ZERO initial messages x (bp/bp.py:43-47), which the first
    layer consumes like any later one: (64,32) at iterations 0 / 1 / 5 and (648,1/2) at 3, clamp 10, x drawn
    N(0, 2^2) per edge (check-order, masking.py:84-88), fp32 module and .double()."""
    from ldpc_amd.codes import get_code
    rec = {}
    for name, iters_list, B in (("peg64_32", (0, 1, 5), 64), ("wifi648_12", (3,), 16)):
        H = parity.H.astype(np.int64) if name == "peg64_32" else np.asarray(get_code(name)[0], np.int64)
        enc = Encoder(H)
        rng = np.random.default_rng(4040 + H.shape[1])
        cw = enc.encode(rng.integers(0, 2, size=(B, enc.k)))
        llr = bpsk_awgn_llr(cw.astype(np.float64), 2.0, enc.k / H.shape[1], rng)
        E = int(H.sum())
        x = (2.0 * rng.standard_normal((B, E))).astype(np.float32)
        rec[f"{name}_llr"] = llr
        rec[f"{name}_x"] = x
        for iters in iters_list:
            model = BeliefPropagation(H, iters)
            model.eval()
            with torch.no_grad():
                p32 = model(torch.tensor(x), torch.tensor(llr), 10.0).numpy()
                m64 = model.double()
                p64 = m64(torch.tensor(x, dtype=torch.float64), torch.tensor(llr, dtype=torch.float64), 10.0).numpy()
            rec[f"{name}_it{iters}_p1_f32"] = p32.astype(np.float32)
            rec[f"{name}_it{iters}_p1_f64"] = p64
            print("x0", name, iters, "ref f32 vs f64 |dp1| max", float(np.abs(p32 - p64).max()), flush=True)
    np.savez_compressed(os.path.join(HERE, "bp_x0.npz"), clamp=10.0, **rec)


def gen_zeros():
    """bp_zeros.npz: LLRs with CLUSTERED exact zeros (erasures): in a third of the checks, two or three of the
    check's variables get an LLR of exactly +0 or -0, the rest BPSK/AWGN values at 2 dB — the s = +-0 case of the
    first VC layer (bp_vc.py:27 gives tanh(0) = 0, so bp_cv.py's product is exactly 0 for every other edge of such
    a check) with several zeros per check row and per variable.  (64,32) and (648,1/2), 1 / 2 / 3 / 5 iterations,
    clamp 10 and 20, the fp32 module and .double(): p1 and z (run_ref_z)."""
    from ldpc_amd.codes import get_code
    rec = {}
    for name, B in (("peg64_32", 64), ("wifi648_12", 16)):
        H = parity.H.astype(np.int64) if name == "peg64_32" else np.asarray(get_code(name)[0], np.int64)
        m, n = H.shape
        enc = Encoder(H)
        rng = np.random.default_rng(7070 + n)
        cw = enc.encode(rng.integers(0, 2, size=(B, enc.k)))
        llr = bpsk_awgn_llr(cw.astype(np.float64), 2.0, enc.k / n, rng)
        nz = 0
        for b in range(B):
            for c in rng.choice(m, size=m // 3, replace=False):
                cols = np.flatnonzero(H[c])
                for v in rng.choice(cols, size=min(len(cols), int(rng.integers(2, 4))), replace=False):
                    llr[b, v] = np.float32(-0.0) if rng.random() < 0.5 else np.float32(0.0)
                    nz += 1
        rec[f"{name}_llr"] = llr
        rec[f"{name}_codeword"] = cw.astype(np.uint8)
        for iters in (1, 2, 3, 5):
            for clamp in (10.0, 20.0):
                tag = f"{name}_it{iters}_cl{int(clamp)}"
                p32, z32 = run_ref_z(H, iters, clamp, llr)
                p64, z64 = run_ref_z(H, iters, clamp, llr, double=True)
                rec[f"{tag}_p1_f32"] = p32.astype(np.float32)
                rec[f"{tag}_z_f32"] = z32.astype(np.float32)
                rec[f"{tag}_p1_f64"] = p64
                rec[f"{tag}_z_f64"] = z64
                print("zeros", tag, "zero LLRs", int((llr == 0).sum()), "exact-zero z (f32/f64):",
                      int((z32 == 0).sum()), int((z64 == 0).sum()), "bit errors:",
                      int((np.round(p32) != cw).sum()), flush=True)
    np.savez_compressed(os.path.join(HERE, "bp_zeros.npz"), **rec)


if __name__ == "__main__":
    parts = sys.argv[1:] or ["bp", "adc", "weighted", "wifi", "x0", "wifilong", "wificlamp", "wificlampb32",
                             "wifi1944c2", "e2e648", "e2eq", "zeros"]
    for part in parts:
        {"bp": gen_bp, "adc": gen_adc, "weighted": gen_weighted, "wifi": gen_wifi_sp, "x0": gen_x0,
         "wifilong": gen_wifi_sp_long,
         "wificlamp": lambda: gen_wifi_sp_long(WIFI_SP_CLAMPS, clamp_tag=True),
         "wificlampb32": gen_wifi_clamp_f32bound, "wifi1944c2": gen_wifi1944_c2, "e2e648": gen_e2e648, "e2eq": gen_e2e_quantized,
         "zeros": gen_zeros}[part]()
    print("done")
