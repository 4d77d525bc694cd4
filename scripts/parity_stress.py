"""Randomised parity sweep on the GPU, time-budgeted: random code, algorithm, parameters, iteration count, batch
size, Eb/N0, erasures and LLR scale per trial, each decoded through the product path and compared with the checker
— bit for bit:
  min-sum           bits, z and iterations used vs oracle.ms_f32 (oracle/ldpc_oracle.c)
  5-bit min-sum     bits, z = app / 2 (by value: the integer posteriors' zero has no sign) and iterations used
                    vs oracle.qms
  fp64 tanh-SP      (--extended) z within 1e-8 relative and bits vs oracle.sp_f64 on the codewords it decodes
                    (decoding failures are chaotic over tens of iterations: not compared, see below)
  tanh-SP           (1) bits, z and iterations used bit for bit vs the generic CSR kernels (the QC kernels'
                    arithmetic is the generic path's, operation for operation, and both apply the a == 1 rule to
                    exactly the codewords whose LLRs hold an exact zero — DESIGN.md §3.5); (2) against the
                    specification, oracle.sp_f32(stable=True), on the codewords the oracle decodes: bits equal, z
                    within 1e-5 relative (scale max(1, |z|)) or, failing that, no further from the reference's fp64
                    than the reference's own fp32 module is (floor 1e-5; growing x1.11 per iteration a codeword
                    takes past the 20th to converge: spec_check), iterations used equal up to threshold ties, and every z the oracle gives as exactly 0 in a codeword with an exact-zero LLR
                    (the rule's outputs) exactly 0 here too.  Decoding failures follow a chaotic fp32 trajectory and
                    are held to (1).
A test-infrastructure script (the oracle is the checker here, never the thing measured).  Prints one line per
kernel path and writes a JSON summary; a mismatching trial's inputs go to OUT/stress_fail_<n>.npz.

    python scripts/parity_stress.py --seconds 420 --out gpurun_out/stress
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "ldpc-sims_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import ldpc_amd  # noqa: E402
import oracle  # noqa: E402
from ldpc_amd.codes import Encoder, IRAEncoder, get_code  # noqa: E402

CODES = ["wifi648_12", "wifi648_23", "wifi648_34", "wifi648_56", "wifi1296_12", "wifi1296_23", "wifi1296_34",
         "wifi1296_56", "wifi1944_12", "wifi1944_23", "wifi1944_34", "wifi1944_56", "peg64_32", "dvbs2_12", "dvbs2s_12"]


GROWTH = 1.11  # per-iteration growth of an fp32 rounding difference on a wandering codeword (measured)


def spec_check(H, x, cw, iters, clamp, es, r, worst=None):
    """tanh-SP against its specification (the oracle's (D, S) form, oracle.sp_f32 stable=True) on the codewords the
    oracle decodes: None when they meet it, else a dict saying how they do not.

    Two fp32 evaluations of the same iteration map differ by the transcendentals' ulps (v_exp / v_log against
    exp2f / log2f), and BP amplifies any rounding while a codeword wanders before it converges: the
    oracle's own fp32 is up to ~3e-4 from fp64 on codewords that converge late (round 6, seed 211).  So, per decoded
    codeword: z within 1e-5 relative of the oracle, or else no further from the reference's exact arithmetic
    (oracle.sp_f64 with the fp32 p bound, same iteration count) than the reference's own fp32 module is
    (oracle.sp_f32 stable=False), with north_star's 1e-5 as the floor, that allowance growing by GROWTH per
    iteration a codeword takes past the 20th to converge (the measured amplification); bits equal; iterations used equal,
    except where the two stop at different iterations because a decision sits on the threshold (the oracle run for
    the GPU's count gives the GPU's bits wherever |z| > 1e-4; z compared at that count) or the stopping iteration is
    not determined at fp32 precision (the reference's own fp32 form stops elsewhere than the oracle: bits only);
    and every exact zero of the a == 1 rule reproduced.  `worst` (a list) collects (GPU distance / allowed) of the rows
    that needed the fp64 comparison."""
    ref = oracle.sp_f32(H, x, iters, clamp, early_stop=es, stable=True)
    decoded = (ref["bits"] == cw).all(1)
    if not decoded.any():
        return None
    gb, gz, gu = (r["bits"].cpu().numpy(), r["soft"].cpu().numpy(), r["iters_used"].cpu().numpy())
    bad = {}
    oz, ob = ref["z"].copy(), ref["bits"].copy()
    moved = decoded & (gu != ref["iters_used"])
    skip = np.zeros(len(x), bool)
    for c in np.nonzero(moved)[0]:
        # the GPU and the oracle stop at different iterations.  A decision sitting on the threshold (the oracle run
        # for the GPU's count gives the GPU's bits wherever |z| > 1e-4): compare z at that count.  Otherwise the
        # stopping iteration is not determined at fp32 precision when the reference's own fp32 form stops elsewhere
        # than the oracle's (a codeword still wandering when it converges): bits only.
        o = oracle.sp_f32(H, x[c:c + 1], int(gu[c]), clamp, stable=True)
        differ = o["bits"][0] != gb[c]
        if (np.abs(o["z"][0][differ]) > 1e-4).any():
            r32 = oracle.sp_f32(H, x[c:c + 1], iters, clamp, early_stop=True, stable=False)["iters_used"][0]
            if r32 == ref["iters_used"][c]:
                bad["iters_rows"] = bad.get("iters_rows", 0) + 1
            skip[c] = True                        # bits only: the GPU's must be the transmitted codeword too
            continue
        oz[c], ob[c] = o["z"][0], gb[c]
    if not np.array_equal(gb[decoded], ob[decoded]):
        bad["bits_rows"] = int((gb[decoded] != ob[decoded]).any(1).sum())
    rel = (np.abs(gz - oz) / np.maximum(np.abs(oz), 1.0)).max(1)
    for c in np.nonzero(decoded & ~skip & (rel > 1e-5))[0]:
        # past 1e-5 of the oracle: held to exact arithmetic instead — the GPU no further from the reference's fp64
        # (oracle.sp_f64, fp32 p bound, same iteration count) than the reference's own fp32 operations are
        # (oracle.sp_f32 stable=False), north_star's 1e-5 where that is larger (tests/softparity.py's rule)
        it_c = int(gu[c]) if es else iters
        xc = x[c:c + 1]
        o64 = oracle.sp_f64(H, xc.astype(np.float64), it_c, clamp, ceiling="f32")["z"][0]
        r32 = oracle.sp_f32(H, xc, it_c, clamp, stable=False)["z"][0]
        sc = np.maximum(np.abs(o64), 1.0)
        e_gpu = float((np.abs(gz[c] - o64) / sc).max())
        e_ref = float((np.abs(r32 - o64) / sc).max())
        # a codeword that wanders before it converges amplifies any fp32 rounding — by x1.11 per iteration on the
        # codeword traced in DESIGN §4 (scripts/trace_failure.py): the allowance grows at that measured rate past
        # iteration 20 (exactly 1e-5 / the module's distance for a codeword converging by then)
        conv = int(gu[c]) if es else int(oracle.sp_f32(H, xc, iters, clamp, early_stop=True, stable=True)["iters_used"][0])
        allowed = max(1e-5, e_ref) * GROWTH ** max(0, conv - 20)
        if worst is not None:
            worst.append(e_gpu / allowed)
        if e_gpu > allowed:
            bad["z_gpu_vs_f64"] = max(bad.get("z_gpu_vs_f64", 0.0), e_gpu)
            bad["z_ref32_vs_f64"] = max(bad.get("z_ref32_vs_f64", 0.0), e_ref)
            bad["converged_at"] = conv
    zr = decoded & (x == 0).any(1)
    if zr.any() and (gz[zr][oz[zr] == 0.0] != 0.0).any():
        bad["rule_zeros"] = int((gz[zr][oz[zr] == 0.0] != 0.0).sum())
    return bad or None


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=420.0)
    ap.add_argument("--trials", type=int, default=0, help="stop after this many trials (0: time budget only)")
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "stress"))
    ap.add_argument("--extended", action="store_true", help="also fp64 tanh-SP vs oracle.sp_f64 (1e-8 relative) "
                    "and host (numpy) inputs through the library's staging path")
    ap.add_argument("--only", default="", help="comma-separated trial numbers: replay just these (same seed), each "
                    "decoded 3 times, to tell a deterministic mismatch from a nondeterministic one")
    a = ap.parse_args(argv)
    os.makedirs(a.out, exist_ok=True)
    rng = np.random.default_rng(a.seed)
    have = set(ldpc_amd.codes.available_codes())
    codes = [c for c in CODES if c in have]
    cache = {}

    def code(name):
        if name not in cache:
            H, _ = get_code(name)
            enc = IRAEncoder(H) if name.startswith("dvbs2") else Encoder(H)
            cache[name] = (H, enc)
        return cache[name]

    decs = {}

    def decoder(name, H):
        if name not in decs:
            decs[name] = ldpc_amd.get_decoder(H)
        return decs[name]

    only = {int(t) for t in a.only.split(",") if t}
    stats, fails, t0, trial = {}, [], time.time(), 0
    spec_worst = []  # tanh-SP: GPU distance / allowed, for the rows compared through fp64 (spec_check)
    last = t0
    while ((time.time() - t0 < a.seconds and (not a.trials or trial < a.trials)) if not only
           else (trial < max(only))):
        trial += 1
        name = codes[rng.integers(len(codes))]
        H, enc = code(name)
        big = name.startswith("dvbs2")
        algos = ("minsum", "qminsum", "tanh") if name.startswith("wifi") else ("minsum", "tanh")  # 5-bit: QC only
        if a.extended:
            algos = algos + ("tanh64",)
        algo = "minsum" if big else algos[rng.integers(len(algos))]
        B = int(rng.integers(1, 13 if big else 300))
        iters = int(rng.integers(0, 21 if big else 51))
        es = bool(rng.integers(2))
        ebn0 = float(rng.uniform(-1.0, 6.0))
        cw = enc.encode(rng.integers(0, 2, size=(B, enc.k)))
        sigma = np.sqrt(1.0 / (2 * 0.5 * 10 ** (ebn0 / 10)))
        x = (-2.0 * ((1.0 - 2.0 * cw) + sigma * rng.standard_normal(cw.shape)) / sigma**2).astype(np.float32)
        if rng.random() < 0.2:
            x[rng.random(x.shape) < 0.05] = 0.0                   # erasures
        if rng.random() < 0.1:
            x *= np.float32(10.0 ** rng.uniform(-3, 6))           # LLR scale extremes
        if only and trial not in only:       # replay: the same draws as the recorded run, no GPU work
            if a.extended and algo in ("minsum", "qminsum"):
                rng.random()
            if algo == "minsum":
                rng.choice([6.0, 20.0, 100.0]), rng.choice([1.0, 0.75, 0.8125]), rng.choice([0.0, 0.0, 0.5])
            elif algo == "qminsum":
                rng.choice([0.5, 1.0, 2.0]), rng.choice([0, 0, 1])
            else:
                rng.choice([10.0, 20.0])
            continue
        desc = dict(trial=trial, code=name, algo=algo, B=B, iters=iters, early_stop=es, ebn0=round(ebn0, 3))
        if only:
            print("replay", json.dumps(desc), flush=True)
        dec = decoder(name, H)
        xg = torch.from_numpy(x).cuda()
        host = bool(a.extended and algo in ("minsum", "qminsum") and rng.random() < 0.3)
        if host:                              # numpy in -> numpy out through the library's host staging
            xg = x
            desc.update(host=True)
        if algo == "minsum":
            clamp = float(rng.choice([6.0, 20.0, 100.0]))
            alpha = float(rng.choice([1.0, 0.75, 0.8125]))
            beta = float(rng.choice([0.0, 0.0, 0.5]))
            desc.update(clamp=clamp, alpha=alpha, beta=beta)
            p = dec.params(iters, "minsum", clamp, alpha=alpha, beta=beta, early_stop=es)
            r = dec.decode(xg, iters, algo="minsum", clamp=clamp, alpha=alpha, beta=beta, early_stop=es, soft="z",
                           want_iters=True)
            ref = oracle.ms_f32(H, x, iters, clamp, alpha, beta, early_stop=es)
            want = (ref["bits"], ref["z"], ref["iters_used"])
        elif algo == "qminsum":
            qstep = float(rng.choice([0.5, 1.0, 2.0]))
            beta = int(rng.choice([0, 0, 1]))
            desc.update(qstep=qstep, beta=beta)
            p = dec.params(iters, "qminsum", 20.0, beta=float(beta), early_stop=es)
            r = dec.decode(xg, iters, algo="qminsum", qstep=qstep, beta=float(beta), early_stop=es, soft="z",
                           want_iters=True)
            q = np.clip(np.rint(x * (np.float32(1.0) / np.float32(qstep))), -15, 15).astype(np.int8)
            ref = oracle.qms(H, q, iters, 15, 127, beta, early_stop=es)
            want = (ref["bits"], (0.5 * ref["app"]).astype(np.float32), ref["iters_used"])
        elif algo == "tanh64":
            clamp = float(rng.choice([10.0, 20.0]))
            desc.update(clamp=clamp)
            x64 = x.astype(np.float64)
            p = dec.params(iters, "tanh", clamp, precision="f64")
            r = dec.decode(x64, iters, algo="tanh", clamp=clamp, soft="z", precision="f64", want_iters=True)
            ref = oracle.sp_f64(H, x64, iters, clamp)
            want = (ref["bits"], ref["z"], np.full(B, iters, np.int32))
        else:
            clamp = float(rng.choice([10.0, 20.0]))
            desc.update(clamp=clamp, zeros=int((x == 0).sum()), maxabs=float(np.abs(x).max()))
            if only:                          # determinism: three decodes of each path
                outs = {}
                for fg in (False, True):
                    zs = []
                    for _ in range(3):
                        o = dec.decode(xg, iters, algo="tanh", clamp=clamp, early_stop=es, soft="z", force_generic=fg)
                        torch.cuda.synchronize()
                        zs.append(o["soft"].cpu().numpy().view(np.uint32))
                    outs[fg] = zs
                    print(trial, "generic" if fg else "qc", "repeat diffs", [int((zs[0] != zz).sum()) for zz in zs[1:]],
                          flush=True)
                d = outs[False][0] != outs[True][0]
                rows = np.nonzero(d.any(1))[0][:10]
                za, zb = outs[False][0].view(np.float32), outs[True][0].view(np.float32)
                rel = [float(np.max(np.abs(za[k] - zb[k]) / np.maximum(np.abs(zb[k]), 1.0))) for k in rows]
                bb = dec.decode(xg, iters, algo="tanh", clamp=clamp, early_stop=es, force_generic=True)["bits"]
                ok_rows = [bool((bb[k].cpu().numpy() == cw[k]).all()) for k in rows]
                print(trial, "qc vs generic", int(d.sum()), "rows", rows.tolist(), "zeros in those rows",
                      [int((x[k] == 0).sum()) for k in rows], "max rel dz", rel, "decoded", ok_rows, flush=True)
            p = dec.params(iters, "tanh", clamp, early_stop=es)
            r = dec.decode(xg, iters, algo="tanh", clamp=clamp, early_stop=es, soft="z", want_iters=True)
            g = dec.decode(xg, iters, algo="tanh", clamp=clamp, early_stop=es, soft="z", want_iters=True,
                           force_generic=True)
            torch.cuda.synchronize()
            want = (g["bits"].cpu().numpy(), g["soft"].cpu().numpy(), g["iters_used"].cpu().numpy())
            spec_bad = spec_check(H, x, cw, iters, clamp, es, r, spec_worst)
            if spec_bad:
                desc.update(spec=spec_bad)
        torch.cuda.synchronize()
        path = dec.kernel_path(p) + ("/es" if es and algo != "tanh64" else "") + ("/host" if host else "")
        npy = (lambda t: t) if isinstance(r["bits"], np.ndarray) else (lambda t: t.cpu().numpy())
        got = (npy(r["bits"]), npy(r["soft"]), npy(r["iters_used"]))
        # z bit for bit; the 5-bit decoder's posteriors are integers, whose zero has no sign: compared by value
        zv = (lambda u: u) if algo == "qminsum" else (lambda u: u.view(np.uint32))
        ulp = False
        if algo == "tanh64":                  # fp64: the reference's operations
            scale = np.maximum(np.abs(want[1]), 1.0)
            rel = np.abs(got[1] - want[1]) / scale
            # decoded codewords: 1e-8, bits equal.  Decoding failures are not compared: BP on a codeword it cannot
            # decode is chaotic over tens of iterations — the oracle itself, fed one fp64 ulp more, moves z by up to
            # 0.16 relative after 42 iterations on seed 47's trial 1777 (profiles/r05/stress/) — so the device's
            # exp / log ulps against glibc's say nothing there; their size is reported (max_rel_failures)
            decoded = (want[0] == cw).all(1)
            zsame = bool((rel[decoded] <= 1e-8).all())
            if decoded.any() and not decoded.all():
                desc.update(max_rel_failures=float(rel[~decoded].max()))
            got = (np.where(decoded[:, None], got[0], want[0]), got[1], got[2])
            if not zsame:
                bad_rows = np.nonzero((rel > 1e-8).any(1))[0]
                desc.update(max_rel=float(rel.max()), rows_over=len(bad_rows),
                            rows_over_decoded=int(sum((want[0][k] == cw[k]).all() for k in bad_rows)))
            clear = np.abs(want[1]) > 1e-9      # bits where the decision is not within 1e-9 of the threshold
            got = (np.where(clear, got[0], want[0]), got[1], got[2])
        else:
            zsame = np.array_equal(zv(got[1]), zv(want[1]))
        ok = np.array_equal(got[0], want[0]) and zsame and np.array_equal(got[2], want[2])
        if algo == "tanh" and "spec" in desc:
            ok = False
        key = f"{name} {algo} {path}"
        s = stats.setdefault(key, [0, 0, 0, 0])
        s[0] += 1
        s[1] += B
        s[3] += ulp
        if not ok:
            s[2] += 1
            desc.update(path=path, bits_diff=int((got[0] != want[0]).sum()),
                        z_diff=int((zv(got[1]) != zv(want[1])).sum()),
                        iters_diff=int((got[2] != want[2]).sum()))
            fails.append(desc)
            if len(fails) <= 5:
                np.savez_compressed(os.path.join(a.out, f"stress_fail_{len(fails)}.npz"), llr=x,
                                    desc=json.dumps(desc))
            print("MISMATCH", json.dumps(desc), flush=True)
        if time.time() - last > 30:
            last = time.time()
            print(f"{last - t0:.0f} s: {trial} trials, {len(fails)} mismatches", flush=True)
    for k in sorted(stats):
        print(f"{k:48s} trials {stats[k][0]:4d} codewords {stats[k][1]:6d} mismatches {stats[k][2]}"
              + (f"  (ulp-level z: {stats[k][3]})" if stats[k][3] else ""))
    if spec_worst:
        print(f"tanh-SP rows past 1e-5 of the oracle, checked against fp64: {len(spec_worst)}, "
              f"max (distance / allowed) {max(spec_worst):.3f}")
    summary = dict(seconds=round(time.time() - t0, 1), seed=a.seed, trials=trial, mismatches=len(fails),
                   spec_fp64_rows=len(spec_worst), spec_fp64_max_ratio=max(spec_worst) if spec_worst else None,
                   per_path={k: dict(trials=v[0], codewords=v[1], mismatches=v[2], ulp_z_trials=v[3])
                             for k, v in stats.items()},
                   failures=fails[:20])
    with open(os.path.join(a.out, "summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(f"{trial} trials, {len(fails)} mismatches")
    return 1 if fails else 0


if __name__ == "__main__":
    sys.exit(main())
