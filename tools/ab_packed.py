"""A/B on one GPU: C3 probe from the 16-B keys vs packing residues once + probing the packed words
(the N>1 broadcast form).  Prints one JSON line; launch durations from fence-free HIP events.

    python tools/ab_packed.py
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "storage-engines_amd"))
import keygen as kg  # noqa: E402
import seb_bloom as seb  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    ts = [seb.Timer() for _ in range(reps + 1)]
    ts[0].record()
    for r in range(reps):
        fn()
        ts[r + 1].record()
    torch.cuda.synchronize()
    return float(np.median([ts[r].elapsed_ms(ts[r + 1]) for r in range(reps)]))


def main():
    seb.device_check(0)
    n = 10_000_000
    m, k = seb.params(n, 0.01)
    keys = torch.from_numpy(kg.key16(np.arange(n))).cuda()
    words = seb.new_words(m)
    seb.dev_build(seb.dev_keys(keys, n=n, stride=16), words, m, k)
    pk = seb.dev_keys(torch.from_numpy(kg.key16(kg.probe_indices(n))).cuda(), n=n, stride=16)
    out = torch.empty(n, dtype=torch.uint8, device="cuda")
    packed = torch.empty(n, dtype=torch.int64, device="cuda")
    res = {
        "probe_keys_ms": timed(lambda: seb.dev_probe(pk, words, m, k, out)),
        "pack_ms": timed(lambda: seb.dev_pack_residues(pk, m, k, packed)),
        "probe_packed_ms": timed(lambda: seb.dev_probe_packed(packed, n, words, m, k, out)),
        "probe_emit_ms": timed(lambda: seb.dev_probe_emit_packed(pk, words, m, k, out, packed)),
    }
    a = out.clone()
    seb.dev_probe(pk, words, m, k, out)
    torch.cuda.synchronize()
    res["same_answers"] = bool(torch.equal(a, out))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
