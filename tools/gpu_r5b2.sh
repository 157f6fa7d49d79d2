#!/bin/bash
# Round 5: the MultiGet's new ordering (sorted answers + unpermute) and its XCD-contiguous block
# remap (multiget_xcd) against the round-4 library (tools/ab_lib/mg_old), lsm and lsm_wide,
# alternating; then a kernel trace of each new variant.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=gpurun_out/${TAG:-r5b2}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "registry or lsm or multiget" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
OLD=$ROOT/tools/ab_lib/mg_old/libseb_bloom.so
for r in 1 2; do
  for cfg in lsm lsm_wide; do
    SEB_MULTIGET_XCD=0 timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 > $OUT/x0_$cfg.$r.json 2>$OUT/err || exit 1
    SEB_MULTIGET_XCD=1 timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 > $OUT/x1_$cfg.$r.json 2>$OUT/err || exit 1
    SEB_LIB_PATH=$OLD timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 > $OUT/old_$cfg.$r.json 2>$OUT/err || exit 1
  done
done
OUT=$OUT python3 - <<'PY'
import json, glob, os
for f in sorted(glob.glob(os.environ["OUT"] + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f"{os.path.basename(f):22s} {d['value']:9.1f} ms {d['ms_per_step']} {d['parity'][:9]}")
PY
cd /tmp && export TMPDIR=/tmp
for x in 0 1; do
  for cfg in lsm lsm_wide; do
    SEB_MULTIGET_XCD=$x timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof_x${x}_$cfg" -o run --output-format csv -- \
        python3 "$ROOT/bench.py" --config $cfg --steps 10 --warmup 3 > "$ROOT/$OUT/prof_x${x}_$cfg.log" 2>&1 || exit 1
  done
done
