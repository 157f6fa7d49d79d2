"""Per-step host timing of the c2_sharded step (debug helper for bench.py's timed region)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "storage-engines_amd")]
import dist_build as db  # noqa: E402
import keygen as kg  # noqa: E402
import seb_bloom as seb  # noqa: E402

n = 10_000_000
m, k = seb.params(n, 0.01)
keys = torch.from_numpy(kg.key16(np.arange(n))).cuda()
kd = seb.dev_keys(keys, n=n, stride=16)
sb = db.ShardedBuild(m, k, 1, 0, "cuda")
bf, of = db.gpu_fns(seb)
for _ in range(3):
    sb.build(kd, bf, of)
torch.cuda.synchronize()
for j in range(8):
    t0 = time.perf_counter()
    sb.build(kd, bf, of)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"step {j}: issue {1e3 * (t1 - t0):.3f} ms, done {1e3 * (t2 - t0):.3f} ms", flush=True)
w = sb.partial
t0 = time.perf_counter()
bits = seb.words_to_bits(w, m)
t1 = time.perf_counter()
import hashlib  # noqa: E402
hashlib.sha256(bits.tobytes()).hexdigest()
t2 = time.perf_counter()
sb.build(kd, bf, of)
t3 = time.perf_counter()
torch.cuda.synchronize()
t4 = time.perf_counter()
print(f"d2h {1e3 * (t1 - t0):.3f} sha {1e3 * (t2 - t1):.3f} next issue {1e3 * (t3 - t2):.3f} done {1e3 * (t4 - t2):.3f}")


def timed(label, pre):
    pre()
    t0 = time.perf_counter()
    sb.build(kd, bf, of)
    torch.cuda.synchronize()
    print(f"{label}: next step {1e3 * (time.perf_counter() - t0):.3f} ms", flush=True)


timed("sleep 10ms", lambda: time.sleep(0.01))
timed("sleep 50ms", lambda: time.sleep(0.05))
timed("d2h only", lambda: seb.words_to_bits(w, m))
timed("nothing", lambda: None)
timed("d2h + sleep 10ms", lambda: (seb.words_to_bits(w, m), time.sleep(0.01)))
timed("alloc 12MB", lambda: torch.empty(3_000_000, dtype=torch.int32, device="cuda"))


def clear_build():
    seb.dev_clear(sb.partial, m)
    seb.dev_build(kd, sb.partial, m, k)


time.sleep(0.02)
t0 = time.perf_counter()
clear_build()
torch.cuda.synchronize()
print(f"sleep 20ms then dev_clear+build: {1e3 * (time.perf_counter() - t0):.3f} ms", flush=True)
