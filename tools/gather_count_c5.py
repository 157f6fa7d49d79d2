"""Count the table gathers of the C5 multi-filter probe (k_probe_interleaved), offline on the CPU
with the numpy oracle (test infrastructure; bench.py only reads the JSON this writes).

C5: 64 filters of 100K keys (m = 958,506, k = 7, filter f built from key16(f*100000
+ j)), one bit-interleaved table entry (u64, bit f = filter f) per bit position, and a 10M-key
batch (even q present in filter (q/2) mod 64, odd q absent from all).  Per key the kernel walks
the table in 2 MiB slices (2^18 u64 entries, table_slice_shift) and, slice by slice, gathers the
entries of the positions in that slice (positions in index order) while the key's AND of the
entries so far is non-zero (lsm/bloom.go:82-92's early exit, for all 64 filters at once).
Writes profiles/gathers_c2c3.json {"c5": {"probe": {...}}}.

    python tools/gather_count_c5.py [--n 10000000]
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
    nf, per, n = 64, 100_000, a.n
    m, k = bn.params(per, 0.01)
    table = np.zeros(m, dtype=np.uint64)
    for f in range(nf):
        h1, h2 = bn.fnv_fixed(kg.key16(f * per + np.arange(per)))
        bits = bn.build(h1, h2, m, k, None)
        b = np.unpackbits(bits, bitorder="little")[:m].astype(np.uint64)
        table |= b << np.uint64(f)
    shift = 18  # 2 MiB of u64 entries per slice
    nsl = (m + (1 << shift) - 1) >> shift
    gathers = 0
    nonzero = 0
    for c0 in range(0, n, a.chunk):
        q = np.arange(c0, min(n, c0 + a.chunk), dtype=np.int64)
        half = q // 2
        idx = np.where(q % 2 == 0, (half % nf) * per + half // nf, nf * per + q)
        h1, h2 = bn.fnv_fixed(kg.key16(idx))
        pos = bn.positions(h1, h2, m, k).astype(np.int64)  # [keys, 7]
        acc = np.full(len(q), np.uint64(0xFFFFFFFFFFFFFFFF))
        sl = pos >> shift
        for s in range(nsl):
            for j in range(k):
                t = (acc != 0) & (sl[:, j] == s)
                gathers += int(t.sum())
                acc = np.where(t, acc & table[pos[:, j]], acc)
        nonzero += int((acc != 0).sum())
    res = {"n": n, "filters": nf, "m": m, "k": k, "slices": int(nsl), "gathers": gathers,
           "per_key": round(gathers / n, 4), "keys_with_a_maybe": nonzero,
           "source": "tools/gather_count_c5.py (numpy oracle, offline)"}
    out = {}
    if os.path.exists(a.out):
        with open(a.out) as f:
            out = json.load(f)
    out.setdefault("c5", {})["probe"] = res
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
