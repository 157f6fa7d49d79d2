"""Count the filter-word gathers one probe call issues (the probe's real bound is the
gather rate, not HBM bytes).  Offline, on the CPU, with the numpy oracle (test infrastructure; the
bench only reads the JSON this writes): C2 filter, C3 batch (10M keys, 50% present), and for each
key the bit tests MayContain makes before its first clear bit (lsm/bloom.go:82-92), counted
  * in the reference's order (positions 0..6), and
  * in the phased probe's order (launch_probe_phased: the filter cut into np word ranges
    [nwords*p/np, nwords*(p+1)/np); range p's positions are tested, in index order, while the key
    is still alive).
Writes profiles/gathers_c2c3.json: {"c2c3": {"probe": {...}}}.

    python tools/gather_count.py [--n 10000000]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--chunk", type=int, default=1_000_000)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "gathers_c2c3.json"))
    a = ap.parse_args()
    n = a.n
    m, k = bn.params(n, 0.01)
    nwords = (m + 31) // 32
    nbytes = (m + 7) // 8
    np_ranges = max(1, (nbytes + (4 << 20) - 1) // (4 << 20))  # probe_phase_count: one per 4 MiB
    bits = None
    for c0 in range(0, n, a.chunk):
        h1, h2 = bn.fnv_fixed(kg.key16(np.arange(c0, min(n, c0 + a.chunk))))
        bits = bn.build(h1, h2, m, k, bits)
    bounds = [nwords * p // np_ranges for p in range(np_ranges + 1)]
    seq = phased = positives = 0
    for c0 in range(0, n, a.chunk):
        q = np.arange(c0, min(n, c0 + a.chunk))
        h1, h2 = bn.fnv_fixed(kg.key16(kg.probe_indices(n, q)))
        pos = bn.positions(h1, h2, m, k).astype(np.int64)  # [keys, k]
        hit = (bits[pos >> 3] >> (pos & 7)) & 1
        alive = np.ones(len(q), dtype=bool)
        for j in range(k):  # reference order
            seq += int(alive.sum())
            alive &= hit[:, j].astype(bool)
        positives += int(alive.sum())
        alive = np.ones(len(q), dtype=bool)
        word = pos >> 5
        for p in range(np_ranges):  # phased order
            inr = (word >= bounds[p]) & (word < bounds[p + 1])
            for j in range(k):
                t = alive & inr[:, j]
                phased += int(t.sum())
                alive &= ~t | hit[:, j].astype(bool)
        assert np.array_equal(alive, hit.all(axis=1))  # the phased walk answers as MayContain does
    res = {"n": n, "m": m, "k": k, "ranges": np_ranges, "positives": positives,
           "gathers_reference_order": seq, "gathers_phased": phased,
           "per_key_phased": round(phased / n, 4),
           "source": "tools/gather_count.py (numpy oracle, offline)"}
    out = {}
    if os.path.exists(a.out):
        with open(a.out) as f:
            out = json.load(f)
    out.setdefault("c2c3", {})["probe"] = res
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
