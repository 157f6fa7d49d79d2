import sys, os
sys.path.insert(0, '.'); sys.path.insert(0, 'storage-engines_amd')
import numpy as np, torch
import seb_bloom as seb, keygen as kg
from oracle import oracle_c as oc
per, nf = 10000, 8
m, k = oc.params(per, 0.01)
keys = torch.from_numpy(kg.key16(np.arange(nf * per))).cuda()
kd = seb.dev_keys(keys, n=nf * per, stride=16)
for variant in ["plain", "one"]:
    nff = nf if variant == "plain" else 1
    filters = [(seb.new_words(m), m, k) for _ in range(nff)]
    begin = [f * per for f in range(nff + 1)]
    seb.dev_build_many(kd, begin, filters)
    torch.cuda.synchronize()
    for f in range(nff):
        got = seb.words_to_bits(filters[f][0], m)
        ref = oc.build(m, k, kg.key16(f * per + np.arange(per)), per, stride=16)
        diff = np.unpackbits(got ^ ref)
        print(variant, f, "popcount got", np.unpackbits(got).sum(), "ref", np.unpackbits(ref).sum(), "diffbits", diff.sum(),
              "extra", np.unpackbits(got & ~ref).sum())
