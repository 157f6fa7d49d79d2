"""Time seb_dev_probe_emit_packed (the per-step broadcast root's probe) with and without the
compacted phases, 10M keys against the C2 filter; prints ms per call (median of 20)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "storage-engines_amd")]
import torch
import seb_bloom as seb
import keygen as kg

n = 10_000_000
m, k = seb.params(n, 0.01)
words = seb.new_words(m)
seb.dev_build_fresh(seb.dev_keys(torch.from_numpy(kg.key16(np.arange(n))).cuda(), n=n, stride=16), words, m, k)
pk = seb.dev_keys(torch.from_numpy(kg.key16(kg.probe_indices(n))).cuda(), n=n, stride=16)
out = torch.empty(n, dtype=torch.uint8, device="cuda")
packed = torch.empty(n, dtype=torch.int64, device="cuda")
res = {}
for rep in range(2):
    for c in (1, 0):
        with seb.option("probe_compact", c):
            ts = []
            for _ in range(23):
                a, b = seb.Timer(), seb.Timer()
                a.record()
                seb.dev_probe_emit_packed(pk, words, m, k, out, packed)
                b.record()
                torch.cuda.synchronize()
                ts.append(a.elapsed_ms(b))
            res.setdefault(c, []).append(float(np.median(ts[3:])))
print({f"compact{c}": v for c, v in res.items()})
