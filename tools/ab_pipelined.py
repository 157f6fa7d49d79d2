"""A/B on one GPU: the c2c3 step as bench.py runs it (clear + build, probe from the keys) against a
pipelined step (clear + build on stream A, probe of batch j from its packed residues on stream A,
and the packing of batch j+1 on stream B overlapping them).  Same work per step; prints JSON lines.

    python tools/ab_pipelined.py
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "storage-engines_amd")]
import keygen as kg  # noqa: E402
import seb_bloom as seb  # noqa: E402

n = 10_000_000
m, k = seb.params(n, 0.01)
bk = seb.dev_keys(torch.from_numpy(kg.key16(np.arange(n))).cuda(), n=n, stride=16)
pkeys = torch.from_numpy(kg.key16(kg.probe_indices(n))).cuda()
pk = seb.dev_keys(pkeys, n=n, stride=16)
words = seb.new_words(m)
out = torch.empty(n, dtype=torch.uint8, device="cuda")
packed = [torch.zeros(n, dtype=torch.int64, device="cuda") for _ in range(2)]
sa = torch.cuda.current_stream()
sb = torch.cuda.Stream()
ev_packed = [torch.cuda.Event() for _ in range(2)]
ev_used = [torch.cuda.Event() for _ in range(2)]


def plain(j):
    seb.dev_clear(words, m)
    seb.dev_build(bk, words, m, k)
    seb.dev_probe(pk, words, m, k, out)


def pipelined(j):
    b = j % 2
    with torch.cuda.stream(sb):  # pack batch j+1 into the other buffer once step j-1's probe released it
        sb.wait_event(ev_used[1 - b])
        seb.dev_pack_residues(pk, m, k, packed[1 - b], stream=sb)
        ev_packed[1 - b].record(sb)
    seb.dev_clear(words, m)
    seb.dev_build(bk, words, m, k)
    sa.wait_event(ev_packed[b])
    seb.dev_probe_packed(packed[b], n, words, m, k, out)
    ev_used[b].record(sa)


def run(fn, steps=40, warm=5):
    for j in range(warm):
        fn(j)
    torch.cuda.synchronize()
    t0, t1 = seb.Timer(), seb.Timer()
    t0.record()
    for j in range(warm, warm + steps):
        fn(j)
    t1.record()
    torch.cuda.synchronize()
    return t0.elapsed_ms(t1) / steps


with torch.cuda.stream(sb):
    seb.dev_pack_residues(pk, m, k, packed[0], stream=sb)
    ev_packed[0].record(sb)
ref = None
for name, fn in (("plain", plain), ("pipelined", pipelined), ("plain2", plain), ("pipelined2", pipelined)):
    ms = run(fn)
    got = out.cpu().numpy().copy()
    ref = got if ref is None else ref
    print(json.dumps({"variant": name, "ms_per_step": round(ms, 4), "mkeys_s": round(2 * n / ms / 1e3, 1),
                      "answers_equal_plain": bool(np.array_equal(got, ref))}), flush=True)
