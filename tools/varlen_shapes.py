"""Pre-hash cost by key-length shape: builds one filter over variable-length keys of a given
length distribution (random bytes), a few times, so `rocprofv3 --kernel-trace --stats` shows what
k_hash_varlen costs per shape.  Usage: python tools/varlen_shapes.py SHAPE [n]
  zipf  the C4 lengths (keygen.varlen_lengths)       uNN  every key NN bytes
  mixK  C4 lengths capped at K bytes"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "storage-engines_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import keygen as kg  # noqa: E402
import seb_bloom as seb  # noqa: E402

shape = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000_000
if shape == "zipf":
    lens = kg.varlen_lengths(np.arange(n)).astype(np.uint64)
elif shape.startswith("mix"):
    lens = np.minimum(kg.varlen_lengths(np.arange(n)), int(shape[3:])).astype(np.uint64)
else:
    lens = np.full(n, int(shape[1:]), np.uint64)
off = np.zeros(n + 1, np.uint64)
np.cumsum(lens, out=off[1:])
total = int(off[-1])
data = torch.randint(0, 256, (total,), dtype=torch.uint8, device="cuda")
offd = torch.from_numpy(off.view(np.int64)).cuda()
m, k = 95850584, 7
words = seb.new_words(m)
kd = seb.dev_keys(data, offd)
for _ in range(6):
    seb.dev_build(kd, words, m, k)
torch.cuda.synchronize()
print(f"{shape}: n={n} bytes={total} mean={total / n:.2f}")
