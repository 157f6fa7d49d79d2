"""Small-batch build latency (memtable-flush sizes): device-scope atomics (build_algo 1), the
radix-partitioned LDS build (2), the LDS-resident filter with an atomic merge (3), LDS images
merged by a second kernel (4) and the auto choice (0) per key count.
    python tools/small_builds.py  -> one JSON line per (n, path) with the median device time."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "storage-engines_amd")]
import keygen as kg  # noqa: E402
import seb_bloom as seb  # noqa: E402
from oracle import oracle_c as oc  # noqa: E402

for n in (1000, 10_000, 50_000, 75_000, 100_000, 130_000, 250_000, 1_000_000):
    m, k = seb.params(n, 0.01)
    keys = torch.from_numpy(kg.key16(np.arange(n))).cuda()
    kd = seb.dev_keys(keys, n=n, stride=16)
    want = oc.build(m, k, kg.key16(np.arange(n)), n, stride=16)
    words = seb.new_words(m)
    paths = {name: (lambda a=a: (seb.set_option("build_algo", a), seb.dev_build(kd, words, m, k)))
             for name, a in (("atomics", 1), ("bucketed", 2), ("lds", 3), ("images", 4), ("auto", 0))}
    if seb.words_bytes(m) > 160 * 1024:
        del paths["lds"], paths["images"]
    for name, fn in paths.items():
        ts = []
        for it in range(12):
            words.zero_()
            a, b = seb.Timer(), seb.Timer()
            a.record()
            fn()
            b.record()
            ts.append(a.elapsed_ms(b))
        torch.cuda.synchronize()
        ok = bool(np.array_equal(seb.words_to_bits(words, m), want))
        print(json.dumps({"n": n, "m": m, "path": name, "us": round(1e3 * float(np.median(ts[2:])), 2), "bit_exact": ok}),
              flush=True)
    seb.set_option("build_algo", 0)
