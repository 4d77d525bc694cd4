"""BER/BLER-vs-Eb/N0 sweep on the GPU, with the reference evaluators' metrics.

Reproduces what ``evaluate_quantized.py`` / ``evaluate_snr.py`` compute around ``decode_bits``
(``evaluate_quantized.py:83-149``): for each SNR point, random information bits, systematic encoding,
channel, LLRs, decode, then
  * uncoded BER  = mean(|sign-decision(llr) - codeword|) over all n bits   (``:139``; cbits = (sign+1)//2)
  * coded BER    = mean(|bits[:, :k] - codeword[:, :k]|) over the information bits (``:140``)
  * coded BLER   = fraction of codewords with any error over all n bits      (``:141``)
The channel is BPSK/AWGN generated on device (``ldpc_awgn_llr``), distributionally identical to the
reference's QPSK over unitary-DFT OFDM at SNR(dB) = Eb/N0(dB) for rate 1/2.
Results can be written in the reference's ``outputs/ber/*.pkl`` key schema so ``plots.py`` reads them.
Long sweeps resume per SNR point: with ``--checkpoint`` (default ``<out>.points.jsonl`` when ``--out`` is
given) every finished point's world-summed counters are appended as one JSON line keyed by the sweep's
configuration, and a restarted sweep with the same configuration skips the points already recorded.

    python -m ldpc_amd.sweep --code peg64_32 --algo tanh --iters 3 --clamp 20 --snr 0:1:10 --n 65536
    python -m ldpc_amd.sweep --gpus 8 ...                    # 8 rank processes, one GPU each (or torchrun)
    torchrun --nproc-per-node 8 -m ldpc_amd.sweep ...        # shards codewords; one RCCL all-reduce
"""
from __future__ import annotations

import argparse
import json
import os
import pickle
import sys
import time

import numpy as np

from . import _abi
from .api import get_decoder
from .codes import get_code
from .channel import adc_quantize, ofdm_demod, ofdm_tx
from .synth import DeviceEncoder
from .dist import ebn0_sigma, shard_bounds


def code_digest(H) -> str:
    """sha1 over H's shape and its nonzeros in check-major CSR order — the identity of a parity-check
    matrix, whatever its container (dense 0/1 array or SparseCode)."""
    import hashlib
    from .codes import Graph
    g = Graph.from_H(H)
    h = hashlib.sha1()
    h.update(np.asarray([g.m, g.n], np.int64).tobytes())
    h.update(np.ascontiguousarray(g.row_ptr, np.int32).tobytes())
    h.update(np.ascontiguousarray(g.col_idx, np.int32).tobytes())
    return h.hexdigest()


def run(code="wifi648_12", algo="minsum", iters=50, clamp=20.0, alpha=1.0, beta=0.0, snr_db=(0.0,),
        codewords=65536, batch=65536, seed=1, rank=0, world=1, device=0, early_stop=False, qstep=1.0,
        qmax=15, app_max=127, mod="bpsk", ofdm_size=32, adc_bits=None, clip_ratio=2.0, checkpoint=None):
    """Returns dict(snrdb, uncoded_ber, coded_ber, coded_bler, codewords, seconds, resumed_points).

    ``mod``: "bpsk" (BPSK/AWGN LLRs), "qpsk-ofdm" (the reference's chain: modulate_bits, transmit_symbols,
    demodulate_signal), "16qam-ofdm" (16-QAM Gray over OFDM, exact LLRs; not in the reference).  Points
    are Eb/N0 in dB; the OFDM modes transmit at Es/N0 = Eb/N0 * R * bits_per_symbol (R = 1/2 QPSK:
    Es/N0 = Eb/N0, the reference's "SNR").

    ``adc_bits`` (OFDM modes only): also run the received samples through the AGC-clipped ADC
    (``gen_qdata``, ``ofdm_functions.py:118-128``; clip = std(rx of the batch) * ``clip_ratio``) and report
    evaluate_quantized.py's ``*_quantized`` metrics and ``wmse_quantized`` (``:122``) next to the
    unquantized ones.

    ``checkpoint``: a JSON-lines file of finished points (see the module docstring): points recorded there
    for this exact configuration (every argument that shapes the data or the decode, a digest of H, a
    digest of the decoder library, the point's index and value, the world size) are taken from it instead
    of being decoded again; rank 0 appends each newly finished point as soon as its counters are summed
    over the ranks.  Ranks without a process group (world > 1 given by hand) use ``<checkpoint>.rank<r>``."""
    import torch
    H, _ = get_code(code) if isinstance(code, str) else (code, None)
    m, n = H.shape
    k = n - m
    rate = k / n
    dec = get_decoder(H, device)
    lib = _abi.load()
    dev = torch.device("cuda", device)
    enc = DeviceEncoder(H, dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    p = dec.params(iters, algo, clamp, alpha, beta, early_stop, "f32", "p1", qmax, app_max, qstep,
                   device_ptrs=True)
    bmax = min(batch, codewords)
    wsb = dec.workspace_bytes(bmax, p)
    ws = torch.empty((max(wsb, 1),), dtype=torch.uint8, device=dev)
    info = torch.empty((bmax, k), dtype=torch.uint8, device=dev)
    llr = torch.empty((bmax, n), dtype=torch.float32, device=dev)
    bits = torch.empty((bmax, n), dtype=torch.uint8, device=dev)
    unc = torch.zeros((len(snr_db),), dtype=torch.int64, device=dev)
    if adc_bits is not None and mod == "bpsk":
        raise ValueError("adc_bits needs an OFDM modulation (the ADC sees the time-domain samples)")
    qcnt = torch.zeros((len(snr_db), 3), dtype=torch.int64, device=dev)
    qunc = torch.zeros((len(snr_db),), dtype=torch.int64, device=dev)
    wmse = torch.zeros((len(snr_db),), dtype=torch.float64, device=dev)

    def run_shard(i, lo, hi, sigma):
        cnt = torch.zeros(3, dtype=torch.int64, device=dev)
        for s in range(lo, hi, bmax):
            B = min(bmax, hi - s)
            _abi.check(lib.ldpc_random_bits(info.data_ptr(), B, k, seed * 7919 + i, s, st))
            cw = enc.encode(info[:B])
            if mod == "bpsk":
                _abi.check(lib.ldpc_awgn_llr(cw.data_ptr(), llr.data_ptr(), B, n, sigma, seed * 104729 + i, s, st))
            else:
                bps = 2 if mod == "qpsk-ofdm" else 4
                esn0 = 10.0 ** (snr_db[i] / 10.0) * rate * bps
                stream = cw.view(-1)
                blk = bps * ofdm_size
                if stream.numel() % blk:  # pad the bit stream to whole OFDM blocks (extra symbols dropped)
                    stream = torch.cat([stream, torch.zeros(blk - stream.numel() % blk, dtype=torch.uint8, device=dev)])
                rx = ofdm_tx(stream, ofdm_size, bps, esn0, seed * 104729 + i, s * n // bps)
                llr[:B].copy_(ofdm_demod(rx, ofdm_size, bps, esn0)[:B * n].view(B, n))
            unc[i] += ((llr[:B] > 0).to(torch.uint8) != cw).sum()      # (np.sign(llr)+1)//2 decisions
            _abi.check(lib.ldpc_decode_ex(dec._h, llr.data_ptr(), B, p, bits.data_ptr(), None, None,
                                          ws.data_ptr(), wsb, st))
            _abi.check(lib.ldpc_count_errors(bits.data_ptr(), cw.data_ptr(), B, n, k, cnt.data_ptr(), st))
            if adc_bits is not None:
                ql = ofdm_demod(adc_quantize(rx, adc_bits, clip_ratio=clip_ratio), ofdm_size, bps, esn0)[:B * n].view(B, n)
                qunc[i] += ((ql > 0).to(torch.uint8) != cw).sum()
                lv = llr[:B].double()
                wmse[i] += ((ql.double() - lv) ** 2 / (lv.abs() + 10e-4)).sum()
                ql = ql.contiguous()
                _abi.check(lib.ldpc_decode_ex(dec._h, ql.data_ptr(), B, p, bits.data_ptr(), None, None,
                                              ws.data_ptr(), wsb, st))
                _abi.check(lib.ldpc_count_errors(bits.data_ptr(), cw.data_ptr(), B, n, k, qcnt[i].data_ptr(), st))
        return cnt.cpu().numpy()

    from .dist import allreduce_counts
    config = dict(code=code if isinstance(code, str) else "custom", algo=algo, iters=iters,
                  clamp=clamp, alpha=alpha, beta=beta, early_stop=early_stop, mod=mod,
                  adc_bits=adc_bits, clip_ratio=clip_ratio if adc_bits is not None else None)
    import torch.distributed as dist
    # counters summed over ranks only inside a process group; without one (tests: rank/world given by hand)
    # each rank keeps its own shard's counts, and its checkpoint records are its own (rank in the key)
    reduced = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    # the key names H itself (a digest of its shape and nonzeros: two custom matrices never share points) and
    # the decoder build (a digest of the loaded library: a rebuilt decoder never resumes old arithmetic)
    fp = dict(config, h_digest=code_digest(H), library=_abi.library_digest(), qstep=qstep, qmax=qmax,
              app_max=app_max, ofdm_size=ofdm_size, codewords=codewords, batch=batch, seed=seed, world=world,
              snr_db=[float(x) for x in snr_db])
    if not reduced and world > 1:
        fp["rank"] = rank
        if checkpoint:  # ranks outside a process group write at once: each gets a file of its own
            checkpoint = f"{checkpoint}.rank{rank}"
    P = len(snr_db)
    cnt = torch.zeros((P, 3), dtype=torch.int64, device=dev)
    # points finished by an earlier run of this configuration: rank 0 reads the checkpoint, the others learn
    # which points to skip through the same all-reduce (they contribute zeros)
    loaded = torch.zeros((P, 1 + 3 + 1 + 3 + 1 + 1), dtype=torch.float64, device=dev)  # done, cnt, unc, qcnt, qunc, wmse
    writer = rank == 0 or not reduced
    if checkpoint and writer and os.path.exists(checkpoint):
        for line in open(checkpoint):
            try:
                rec = json.loads(line)
            except ValueError:
                continue  # a line cut short by an interrupted write
            i = rec.get("i", -1)
            if rec.get("config") == fp and 0 <= i < P and rec.get("snr") == float(snr_db[i]):
                loaded[i] = torch.tensor([1.0, *rec["counts"], rec["uncoded"], *rec["counts_quantized"],
                                          rec["quantized_uncoded"], rec["wmse"]], dtype=torch.float64)
    allreduce_counts(loaded)
    if checkpoint and writer and os.path.exists(checkpoint) and os.path.getsize(checkpoint):
        with open(checkpoint, "rb+") as f:    # a torn last line (interrupted write): end it before appending
            f.seek(-1, os.SEEK_END)
            if f.read(1) != b"\n":
                f.write(b"\n")
    t0 = time.perf_counter()
    resumed = []
    for i in range(P):
        if loaded[i, 0].item() > 0:
            resumed.append(i)
            if writer:
                cnt[i] = loaded[i, 1:4].to(torch.int64)
                unc[i] = loaded[i, 4].to(torch.int64)
                qcnt[i] = loaded[i, 5:8].to(torch.int64)
                qunc[i] = loaded[i, 8].to(torch.int64)
                wmse[i] = loaded[i, 9]
            continue
        lo, hi = shard_bounds(codewords, rank, world)
        if hi > lo:
            cnt[i] += torch.as_tensor(run_shard(i, lo, hi, ebn0_sigma(snr_db[i], rate)), device=dev)
        pt = torch.cat([cnt[i].double(), unc[i:i + 1].double(), qcnt[i].double(), qunc[i:i + 1].double(),
                        wmse[i:i + 1]])
        allreduce_counts(pt)  # this point's counters summed over the ranks
        if writer:
            cnt[i], unc[i], qcnt[i], qunc[i], wmse[i] = (pt[0:3].to(torch.int64), pt[3].to(torch.int64),
                                                         pt[4:7].to(torch.int64), pt[7].to(torch.int64), pt[8])
            if checkpoint:
                rec = dict(config=fp, i=i, snr=float(snr_db[i]), counts=[int(v) for v in pt[0:3].tolist()],
                           uncoded=int(pt[3].item()), counts_quantized=[int(v) for v in pt[4:7].tolist()],
                           quantized_uncoded=int(pt[7].item()), wmse=float(pt[8].item()))
                with open(checkpoint, "a") as f:
                    f.write(json.dumps(rec) + "\n")
                    f.flush()
                    os.fsync(f.fileno())
        else:
            for t in (cnt[i], unc[i:i + 1], qcnt[i], qunc[i:i + 1], wmse[i:i + 1]):
                t.zero_()  # rank 0 holds the point's totals; the closing all-reduce hands them to everyone
    if reduced:
        for t in (cnt, unc, qcnt, qunc, wmse):
            allreduce_counts(t)
    secs = time.perf_counter() - t0
    c = cnt.cpu().numpy().astype(np.float64)
    out = dict(snrdb=np.asarray(snr_db, dtype=np.float64),
               uncoded_ber=unc.cpu().numpy() / (c[:, 2] * n),
               coded_ber=c[:, 0] / (c[:, 2] * k),
               coded_bler=c[:, 1] / c[:, 2],
               codewords=c[:, 2].astype(np.int64), seconds=secs, resumed_points=resumed, config=config)
    if adc_bits is not None:
        q = qcnt.cpu().numpy().astype(np.float64)
        out.update(uncoded_ber_quantized=qunc.cpu().numpy() / (c[:, 2] * n),
                   coded_ber_quantized=q[:, 0] / (c[:, 2] * k), coded_bler_quantized=q[:, 1] / c[:, 2],
                   wmse_quantized=wmse.cpu().numpy() / (c[:, 2] * n))
    return out


# every key evaluate_quantized.py:155-172 writes and plots.py:12-27 reads, in the reference's order
PKL_KEYS = ("snrdb", "uncoded_ber", "coded_ber", "coded_bler",
            "uncoded_ber_nn", "coded_ber_nn", "coded_bler_nn",
            "uncoded_ber_quantized", "coded_ber_quantized", "coded_bler_quantized",
            "wmse_nn", "wmse_quantized")


def ebn0_at(snr_db, curve, level):
    """Eb/N0 (dB) where a monotone error-rate curve crosses ``level``: linear interpolation of log10(rate)
    between the two grid points that bracket it (points with rate 0 are dropped).  None if not bracketed."""
    x = np.asarray(snr_db, np.float64)
    y = np.asarray(curve, np.float64)
    keep = y > 0
    x, ly, t = x[keep], np.log10(y[keep]), np.log10(level)
    for i in range(len(x) - 1):
        if ly[i] >= t >= ly[i + 1] and ly[i] != ly[i + 1]:
            return float(x[i] + (ly[i] - t) * (x[i + 1] - x[i]) / (ly[i] - ly[i + 1]))
    return None


def ebn0_offset_db(snr_db, curve, ref_curve, level):
    """Horizontal distance (dB) of ``curve`` from ``ref_curve`` at error rate ``level``: positive = curve
    needs more Eb/N0 than the reference for the same rate.  The quantity north_star bounds by +-0.05 dB."""
    a, b = ebn0_at(snr_db, curve, level), ebn0_at(snr_db, ref_curve, level)
    return None if a is None or b is None else a - b


def save(result: dict, path: str):
    """``.pkl``: the reference's schema — all 12 keys of ``evaluate_quantized.py:155-172`` as float64
    numpy arrays of one entry per SNR point, so ``plots.py`` reads the file unchanged.  The ``*_nn`` keys
    (the NN LLR estimator, out of scope here) and, for a sweep run without ``--adc-bits``, the
    ``*_quantized`` keys are NaN arrays of the right length (matplotlib skips NaN points).
    ``.json``: every result field as plain lists."""
    if path.endswith(".pkl"):
        npts = len(np.asarray(result["snrdb"]))
        keep = {kk: (np.asarray(result[kk], dtype=np.float64) if kk in result else np.full(npts, np.nan))
                for kk in PKL_KEYS}
        with open(path, "wb") as f:
            pickle.dump(keep, f)
    else:
        with open(path, "w") as f:
            json.dump({kk: (v.tolist() if isinstance(v, np.ndarray) else v) for kk, v in result.items()}, f, indent=1)


def _parse_points(s):
    lo, st, hi = (float(x) for x in s.split(":"))
    return list(np.round(np.arange(lo, hi + 1e-9, st), 6))


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--code", default="wifi648_12")
    ap.add_argument("--algo", default="minsum")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--clamp", type=float, default=20.0)
    ap.add_argument("--alpha", type=float, default=1.0)
    ap.add_argument("--beta", type=float, default=0.0)
    ap.add_argument("--snr", default="0:0.5:5")
    ap.add_argument("--n", type=int, default=65536, help="codewords per SNR point (all ranks)")
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--early-stop", action="store_true")
    ap.add_argument("--mod", default="bpsk", choices=["bpsk", "qpsk-ofdm", "16qam-ofdm"])
    ap.add_argument("--adc-bits", type=int, default=None, help="also decode through the AGC-clipped ADC")
    ap.add_argument("--clip-ratio", type=float, default=2.0)
    ap.add_argument("--out", default=None, help="results .json or .pkl (reference schema)")
    ap.add_argument("--checkpoint", default=None,
                    help="per-point resume file (JSON lines); default <out>.points.jsonl when --out is given")
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one GPU each); N > 1 without a launcher starts N rank processes itself")
    a = ap.parse_args(argv)
    if a.gpus is not None:
        from .dist import resolve_world, spawn_ranks
        spawn = resolve_world(a.gpus)
        if spawn is not None and spawn > 1:
            pkg_root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
            env = dict(os.environ, PYTHONPATH=os.pathsep.join(
                x for x in (pkg_root, os.environ.get("PYTHONPATH")) if x))
            args = list(sys.argv[1:] if argv is None else argv)
            raise SystemExit(spawn_ranks(["-m", "ldpc_amd.sweep", *args], spawn, env=env))
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # LDPC_BENCH_SHARE_GPU / LDPC_BENCH_BACKEND (as in bench.py) only rehearse N>1 ranks on a 1-GPU box
    # (ranks share cuda:0, counters over gloo); real multi-GPU runs use one GPU per rank and RCCL.
    if os.environ.get("LDPC_BENCH_SHARE_GPU"):
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        backend = os.environ.get("LDPC_BENCH_BACKEND", "nccl")  # nccl == RCCL over xGMI
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    ckpt = a.checkpoint or (a.out + ".points.jsonl" if a.out else None)
    r = run(a.code, a.algo, a.iters, a.clamp, a.alpha, a.beta, _parse_points(a.snr), a.n, a.batch, a.seed,
            rank, world, local, a.early_stop, mod=a.mod, adc_bits=a.adc_bits, clip_ratio=a.clip_ratio, checkpoint=ckpt)
    if rank == 0:
        for i, e in enumerate(r["snrdb"]):
            line = (f"{e:5.2f} dB  uncoded {r['uncoded_ber'][i]:.4e}  coded BER {r['coded_ber'][i]:.4e}  "
                    f"BLER {r['coded_bler'][i]:.4e}  ({r['codewords'][i]} cw)")
            if "coded_ber_quantized" in r:
                line += (f" | ADC uncoded {r['uncoded_ber_quantized'][i]:.4e} BER {r['coded_ber_quantized'][i]:.4e} "
                         f"BLER {r['coded_bler_quantized'][i]:.4e} wmse {r['wmse_quantized'][i]:.4g}")
            print(line)
        print(f"{r['seconds']:.2f} s" + (f" (points {r['resumed_points']} from {ckpt})" if r["resumed_points"] else ""))
        if a.out:
            save(r, a.out)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
