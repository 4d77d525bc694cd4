#!/usr/bin/env python3
"""Emit qc_tables.h: compile-time descriptions of the QC base matrices that get specialised kernels.

    python ldpc-sims_amd/csrc/gen_qc_tables.py > ldpc-sims_amd/csrc/qc_tables.h

Source of truth: ldpc_amd/codes.py (802.11n tables).  Every row lists its non-null block columns in
ascending order (= the reference's check-order edge order within a row, bp/masking.py:84-88).
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from ldpc_amd.codes import wifi_code  # noqa: E402

CODES = [("Wifi648_12", 648, "1/2"), ("Wifi1296_23", 1296, "2/3"), ("Wifi1944_56", 1944, "5/6")]
ASCENT_FRAMES = {"Wifi1296_23"}  # codes that keep the round-1 frame search (lane_frames_ascent)


def lane_frames(base, Z, trials=8000, seed=11):
    """Lane relabelling that maximises zero-shift circulants.

    The kernel may hold variable (j, (z + phi_j) mod Z) in lane z and check (r, (z + psi_r) mod Z) in lane
    z: a pure relabelling (bit-exact), under which circulant (r, j, s) becomes a rotation by
    (s - phi_j + psi_r) mod Z, and rotation 0 needs no lane exchange (two ds_bpermute fewer per iteration).
    Coordinate ascent over (phi, psi) from random spanning-tree starts (a spanning tree of the base graph
    already gives MB + NB - 1 zeros), with random moves along plateaus of equal count (without them the
    ascent stalls early: (648,1/2) 41 -> 44 zeros, (1296,2/3) 36 -> 38).  Only phi reaches the kernel
    (LLR load / bit store index); check labels are internal."""
    import random
    from collections import Counter
    mb, nb = base.shape
    edges = [(i, j, int(base[i, j])) for i in range(mb) for j in range(nb) if base[i, j] >= 0]
    rows = {i: [(j, s) for (ii, j, s) in edges if ii == i] for i in range(mb)}
    cols = {j: [(i, s) for (i, jj, s) in edges if jj == j] for j in range(nb)}
    rng = random.Random(seed)
    best = (sum(1 for e in edges if e[2] == 0), [0] * mb, [0] * nb)
    for _trial in range(trials):
        psi = [rng.randrange(Z) for _ in range(mb)]
        phi = [rng.randrange(Z) for _ in range(nb)]
        order = edges[:]
        rng.shuffle(order)
        seen_r, seen_c = {rng.randrange(mb)}, set()
        grown = True
        while grown:  # a random spanning tree made all-zero
            grown = False
            for (i, j, s) in order:
                if i in seen_r and j not in seen_c:
                    phi[j] = (s + psi[i]) % Z
                    seen_c.add(j)
                    grown = True
                elif j in seen_c and i not in seen_r:
                    psi[i] = (phi[j] - s) % Z
                    seen_r.add(i)
                    grown = True
        for _sweep in range(40):
            for k in rng.sample(range(mb + nb), mb + nb):
                if k < mb:
                    c = Counter((phi[j] - s) % Z for (j, s) in rows[k])
                    top = max(c.values())
                    v = rng.choice([x for x, m in c.items() if m == top])
                    if top > c[psi[k]] or (v != psi[k] and rng.random() < 0.3):
                        psi[k] = v
                else:
                    jj = k - mb
                    c = Counter((s + psi[i]) % Z for (i, s) in cols[jj])
                    top = max(c.values())
                    v = rng.choice([x for x, m in c.items() if m == top])
                    if top > c[phi[jj]] or (v != phi[jj] and rng.random() < 0.3):
                        phi[jj] = v
            cnt = sum(1 for (i, j, s) in edges if (s - phi[j] + psi[i]) % Z == 0)
            if cnt > best[0]:
                best = (cnt, list(psi), list(phi))
    return best


def lane_frames_ascent(base, Z, trials=400, seed=1):
    """The round-1 search (strict ascent, alternating random and spanning-tree starts): kept for (1296,2/3),
    whose packed 5-bit kernel measured 1.2 % faster with these frames (36 zeros) than with 38 (A/B).

    Lane relabelling that maximises zero-shift circulants.

    The kernel may hold variable (j, (z + phi_j) mod Z) in lane z and check (r, (z + psi_r) mod Z) in lane
    z: a pure relabelling (bit-exact), under which circulant (r, j, s) becomes a rotation by
    (s - phi_j + psi_r) mod Z, and rotation 0 needs no lane exchange.  Local search over (phi, psi) from
    random starts (a spanning tree of the base graph already gives MB + NB - 1 zeros).  Only phi reaches
    the kernel (LLR load / bit store index); check labels are internal."""
    import random
    from collections import Counter
    mb, nb = base.shape
    edges = [(i, j, int(base[i, j])) for i in range(mb) for j in range(nb) if base[i, j] >= 0]
    rng = random.Random(seed)
    best = (sum(1 for e in edges if e[2] == 0), [0] * mb, [0] * nb)
    for trial in range(trials):
        psi = [rng.randrange(Z) for _ in range(mb)]
        phi = [rng.randrange(Z) for _ in range(nb)]
        if trial % 2 == 0:  # start from a random spanning tree made all-zero
            order = edges[:]
            rng.shuffle(order)
            seen_r, seen_c = {rng.randrange(mb)}, set()
            grown = True
            while grown:
                grown = False
                for (i, j, s) in order:
                    if i in seen_r and j not in seen_c:
                        phi[j] = (s + psi[i]) % Z
                        seen_c.add(j)
                        grown = True
                    elif j in seen_c and i not in seen_r:
                        psi[i] = (phi[j] - s) % Z
                        seen_r.add(i)
                        grown = True
        for _sweep in range(30):
            changed = False
            for k in rng.sample(range(mb + nb), mb + nb):
                if k < mb:
                    c = Counter((phi[j] - s) % Z for (i, j, s) in edges if i == k)
                    v = max(c.items(), key=lambda a: a[1])[0]
                    if c[v] > c[psi[k]]:
                        psi[k], changed = v, True
                else:
                    jj = k - mb
                    c = Counter((s + psi[i]) % Z for (i, j, s) in edges if j == jj)
                    v = max(c.items(), key=lambda a: a[1])[0]
                    if c[v] > c[phi[jj]]:
                        phi[jj], changed = v, True
            if not changed:
                break
        cnt = sum(1 for (i, j, s) in edges if (s - phi[j] + psi[i]) % Z == 0)
        if cnt > best[0]:
            best = (cnt, list(psi), list(phi))
    return best


def emit(name, q):
    mb, nb = q.base.shape
    rows = [[(j, int(q.base[r, j])) for j in range(nb) if q.base[r, j] >= 0] for r in range(mb)]
    nzero, psi, phi = (lane_frames_ascent if name in ASCENT_FRAMES else lane_frames)(q.base, q.Z)
    maxdc = max(len(r) for r in rows)
    pad = lambda xs: xs + [-1] * (maxdc - len(xs))
    # Z > 64: the lifting index is split into S slots of ZL = Z / S <= 32 lanes (one wave per slot, two
    # codewords per wave; qc.hip k_qc_*_sl exchange through LDS)
    S = 1 if q.Z <= 64 else next(s for s in range(2, q.Z + 1) if q.Z % s == 0 and q.Z // s <= 32)
    out = [f"struct {name} {{",
           f"    static constexpr int MB = {mb}, NB = {nb}, Z = {q.Z}, MAXDC = {maxdc}, S = {S};",
           f"    static constexpr int DEG[MB] = {{{', '.join(str(len(r)) for r in rows)}}};",
           "    static constexpr int COL[MB][MAXDC] = {"]
    out += ["        {" + ", ".join(str(x) for x in pad([j for j, _ in r])) + "}," for r in rows]
    out += ["    };", "    static constexpr int SH[MB][MAXDC] = {"]
    out += ["        {" + ", ".join(str(x) for x in pad([s for _, s in r])) + "}," for r in rows]
    out += ["    };",
            f"    // lane frames: {nzero} of {sum(len(r) for r in rows)} circulants become rotation 0 (was "
            f"{sum(1 for r in rows for _, s in r if s == 0)})",
            f"    static constexpr int PHI[NB] = {{{', '.join(str(x) for x in phi)}}};",
            "    static constexpr int SHR[MB][MAXDC] = {"]
    out += ["        {" + ", ".join(str(x) for x in pad([(s - phi[j] + psi[r]) % q.Z for j, s in rows[r]])) + "},"
            for r in range(mb)]
    out += ["    };", f"    static constexpr const char* NAME = \"{q.name}\";", "};", ""]
    return "\n".join(out)


def main():
    print("// Generated by gen_qc_tables.py from ldpc_amd/codes.py — do not edit.")
    print("#pragma once\n")
    print("namespace ldpc {\n")
    for name, n, r in CODES:
        print(emit(name, wifi_code(n, r)))
    print("}  // namespace ldpc")


if __name__ == "__main__":
    main()
