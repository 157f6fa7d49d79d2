#!/bin/bash
# C5 slice-size A/B: product (2 MB slices) vs sl22 (4 MB) vs sl20 (1 MB), alternating, 3 rounds
OUT=gpurun_out/r6sl; mkdir -p $OUT
for r in 1 2 3; do
  for name in product sl22 sl20; do
    lib=tools/ab_lib/$name/libseb_bloom.so; [ $name = product ] && lib=storage-engines_amd/lib/libseb_bloom.so
    SEB_LIB_PATH=$lib timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline --no-host-inclusive --no-secondary > $OUT/$name.$r.json 2> $OUT/$name.$r.err || exit 1
  done
done
python3 - <<'PY'
import glob, json, os
rows = {}
for f in sorted(glob.glob("gpurun_out/r6sl/*.json")):
    name, r, _ = os.path.basename(f).split(".")
    d = json.loads(open(f).read().strip().splitlines()[-1])
    rows.setdefault(name, []).append((d["ms_per_step"], d["parity"][:9]))
for name, v in sorted(rows.items()):
    print(f"{name:8s}", " ".join(f"{ms:.4f}" for ms, _ in v), {p for _, p in v})
PY
