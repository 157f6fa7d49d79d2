#!/bin/bash
# Round 5: MultiGet unpermute per chunk through LDS (many buckets) vs the per-key gather: parity of
# both, then kernel traces of lsm / lsm_wide with each forced (SEB_MG_CHUNKED_MIN 0 / 100000).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=gpurun_out/r5i
mkdir -p $OUT
for cm in 0 100000; do
  SEB_MG_CHUNKED_MIN=$cm timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
      tests/test_gpu_parity.py -k "registry or lsm or multiget" > $OUT/tests_$cm.log 2>&1 || { tail -40 $OUT/tests_$cm.log; exit 1; }
  tail -1 $OUT/tests_$cm.log
done
cd /tmp && export TMPDIR=/tmp
for cm in 0 100000; do
  for cfg in lsm lsm_wide; do
    SEB_MG_CHUNKED_MIN=$cm timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof_c${cm}_$cfg" -o run --output-format csv -- \
        python3 "$ROOT/bench.py" --config $cfg --steps 10 --warmup 3 > "$ROOT/$OUT/prof_c${cm}_$cfg.log" 2>&1 || exit 1
  done
done
