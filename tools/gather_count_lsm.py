"""Count the filter-word gathers of one registry MultiGet call (bench.py --config lsm / lsm_wide),
offline on the CPU with the numpy oracle (test infrastructure; the bench only reads the JSON this
writes).  Per key, LSM.Get's walk (lsm/lsm.go:168-198): every L0 filter, then per level the
covering file's filter, each tested with MayContain's early exit (lsm/bloom.go:82-92): a test
costs one gather per position up to and including the first clear bit.
The L0 files that share (m, k) are tested as one group through the registry's interleaved table
(multiget_l0_group): one gather per position while any member is still alive; "gathers" counts
that, "gathers_per_file" the walk with one MayContain per L0 file.
Writes profiles/gathers_c2c3.json["lsm" | "lsm_wide"]["probe"].

    python tools/gather_count_lsm.py [--wide]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "storage-engines_amd")]

import keygen as kg  # noqa: E402
from oracle import bloom_np as bn  # noqa: E402


def gathers(bits, h1, h2, m, k):
    """Gathers of MayContain per key (early exit) and its answers."""
    pos = bn.positions(h1, h2, m, k).astype(np.int64)
    hit = ((bits[pos >> 3] >> (pos & 7)) & 1).astype(bool)
    alive = np.ones(len(h1), bool)
    cnt = np.zeros(len(h1), np.int64)
    for j in range(k):
        cnt += alive
        alive &= hit[:, j]
    return cnt, alive


def group_gathers(members, h1, h2):
    """Gathers of the L0 group walk: positions up to the one where the last member dies."""
    m, k = members[0][4], members[0][5]
    pos = bn.positions(h1, h2, m, k).astype(np.int64)
    alive = np.ones((len(h1), len(members)), bool)
    cnt = np.zeros(len(h1), np.int64)
    for j in range(k):
        cnt += alive.any(axis=1)
        for g, f in enumerate(members):
            alive[:, g] &= ((f[3][pos[:, j] >> 3] >> (pos[:, j] & 7)) & 1).astype(bool)
    return cnt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--wide", action="store_true")
    ap.add_argument("--chunk", type=int, default=1_000_000)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "gathers_c2c3.json"))
    a = ap.parse_args()
    lay = kg.LSM_WIDE_LAYOUT if a.wide else kg.LSM_LAYOUT
    files = kg.lsm_files(lay)
    filt = []  # (level, lo_i, hi_i, bits, m, k): key16(2i) for i in the file; range [2*lo_i, 2*hi_i]
    for level, _, idx in files:
        m, k = bn.params(len(idx), 0.01)
        bits = None
        for c0 in range(0, len(idx), a.chunk):
            h1, h2 = bn.fnv_fixed(kg.key16(2 * idx[c0:c0 + a.chunk]))
            bits = bn.build(h1, h2, m, k, bits)
        filt.append((level, int(idx[0]), int(idx[-1]), bits, m, k))
    l0 = [f for f in filt if f[0] == 0]  # insertion order
    shapes = {}
    for f in l0:
        shapes.setdefault((f[4], f[5]), []).append(f)
    group = max(shapes.values(), key=len) if shapes else []
    group = group if len(group) >= 2 else []
    levels = {L: sorted([f for f in filt if f[0] == L], key=lambda f: f[1]) for L in (1, 2, 3, 4)}
    pidx = kg.lsm_probe_indices(lay)
    n = len(pidx)
    total = tests = per_file = 0
    per_level = {}
    for c0 in range(0, n, a.chunk):
        x = pidx[c0:c0 + a.chunk]  # key16(x); key16 sorts as x does
        h1, h2 = bn.fnv_fixed(kg.key16(x))
        for f in l0:
            cnt, _ = gathers(f[3], h1, h2, f[4], f[5])
            per_file += int(cnt.sum())
            tests += len(x)
            if not any(f is g for g in group):
                total += int(cnt.sum())
                per_level[0] = per_level.get(0, 0) + int(cnt.sum())
        if group:
            gc = int(group_gathers(group, h1, h2).sum())
            total += gc
            per_level[0] = per_level.get(0, 0) + gc
        for L, fs in levels.items():
            if not fs:
                continue
            lo = np.array([2 * f[1] for f in fs])
            j = np.searchsorted(lo, x, side="right") - 1  # last file with MinKey <= key
            hi = np.array([2 * f[2] for f in fs])
            cov = (j >= 0) & (x <= hi[np.maximum(j, 0)])
            for fi in np.unique(j[cov]):
                sel = cov & (j == fi)
                f = fs[fi]
                cnt, _ = gathers(f[3], h1[sel], h2[sel], f[4], f[5])
                total += int(cnt.sum())
                per_file += int(cnt.sum())
                tests += int(sel.sum())
                per_level[L] = per_level.get(L, 0) + int(cnt.sum())
    res = {"n": n, "files": len(files), "filter_tests": tests, "gathers": total, "gathers_per_file": per_file,
           "l0_group": len(group),
           "per_key": round(total / n, 4), "per_level": per_level,
           "source": "tools/gather_count_lsm.py (numpy oracle, offline)"}
    out = {}
    if os.path.exists(a.out):
        with open(a.out) as f:
            out = json.load(f)
    out.setdefault("lsm_wide" if a.wide else "lsm", {})["probe"] = res
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
