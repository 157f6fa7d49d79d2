#!/bin/bash
# A/B of the current library against tools/ab_lib/prev2 (parity: varlen, c4, registry tests), alternating bench
# runs of CFGS and kernel traces of PCFGS; TAG names gpurun_out/TAG.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=gpurun_out/${TAG:-r5l}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "varlen or c4 or registry or lsm or multiget" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
PREV=$ROOT/tools/ab_lib/prev2/libseb_bloom.so
for r in 1 2; do
  for cfg in ${CFGS:-c4 lsm lsm_wide}; do
    timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline > $OUT/new_$cfg.$r.json 2>$OUT/err || exit 1
    SEB_LIB_PATH=$PREV timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prev_$cfg.$r.json 2>$OUT/err || exit 1
  done
done
OUT=$OUT python3 - <<'PY'
import json, glob, os
for f in sorted(glob.glob(os.environ["OUT"] + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f"{os.path.basename(f):22s} {d['value']:9.1f} ms {d['ms_per_step']} {d.get('build_ms')} {d.get('probe_ms')} {d['parity'][:9]}")
PY
cd /tmp && export TMPDIR=/tmp
for cfg in ${PCFGS:-c4 lsm}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof_$cfg" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > "$ROOT/$OUT/prof_$cfg.log" 2>&1 || exit 1
done
