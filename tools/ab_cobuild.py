"""A/B on one GPU: the c2c3 step as bench.py runs it (a fresh build, then the probe from the keys)
against a step whose probe batch is hashed and packed on a second stream WHILE the filter builds
(the packing needs no filter), then probed from its packed residues once the build is done.  Same
batch and work per step, no cross-step pipelining; answers checked against the plain step and the
golden digest.  Prints JSON lines.

    python tools/ab_cobuild.py
"""
import hashlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "storage-engines_amd")]
import keygen as kg  # noqa: E402
import seb_bloom as seb  # noqa: E402

GOLDEN_C3 = "aba77536fae51d566de525f519cd4c573799880d63000d88a2ce3052d0b90f95"
n = 10_000_000
m, k = seb.params(n, 0.01)
bk = seb.dev_keys(torch.from_numpy(kg.key16(np.arange(n))).cuda(), n=n, stride=16)
pk = seb.dev_keys(torch.from_numpy(kg.key16(kg.probe_indices(n))).cuda(), n=n, stride=16)
words = seb.new_words(m)
out = torch.empty(n, dtype=torch.uint8, device="cuda")
packed = torch.zeros(n, dtype=torch.int64, device="cuda")
sa = torch.cuda.current_stream()
sb = torch.cuda.Stream()
ev_start, ev_packed = torch.cuda.Event(), torch.cuda.Event()


def plain(j):
    seb.dev_build_fresh(bk, words, m, k)
    seb.dev_probe(pk, words, m, k, out)


def cobuild(j):
    ev_start.record(sa)  # the previous step's probe has released `packed`
    with torch.cuda.stream(sb):
        sb.wait_event(ev_start)
        seb.dev_pack_residues(pk, m, k, packed, stream=sb)
        ev_packed.record(sb)
    seb.dev_build_fresh(bk, words, m, k)
    sa.wait_event(ev_packed)
    seb.dev_probe_packed(packed, n, words, m, k, out)


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


ref = None
for name, fn in (("plain", plain), ("cobuild", cobuild), ("plain2", plain), ("cobuild2", cobuild),
                 ("plain3", plain), ("cobuild3", cobuild)):
    out.fill_(7)
    ms = run(fn)
    got = out.cpu().numpy().copy()
    ref = got if ref is None else ref
    print(json.dumps({"variant": name, "ms_per_step": round(ms, 4), "mkeys_s": round(2 * n / ms / 1e3, 1),
                      "answers_equal_plain": bool(np.array_equal(got, ref)),
                      "golden": hashlib.sha256(got.tobytes()).hexdigest() == GOLDEN_C3}), flush=True)
