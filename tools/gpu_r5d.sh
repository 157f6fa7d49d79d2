#!/bin/bash
# Round 5: MultiGet ordering A/B over the number of tiles (SEB_MG_TILES), kernel traces.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=gpurun_out/${TAG:-r5d}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "registry or lsm or multiget" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
SEB_MG_TILES=8192 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "registry or lsm or multiget" > $OUT/tests8192.log 2>&1 || { tail -40 $OUT/tests8192.log; exit 1; }
tail -1 $OUT/tests8192.log
cd /tmp && export TMPDIR=/tmp
for st in ${STAGES:-0 1}; do
  for cfg in lsm lsm_wide; do
    SEB_MULTIGET_XCD=1 SEB_MG_STAGE=0 SEB_MG_TILES=$st timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof_t${st}_$cfg" -o run --output-format csv -- \
        python3 "$ROOT/bench.py" --config $cfg --steps 10 --warmup 3 > "$ROOT/$OUT/prof_t${st}_$cfg.log" 2>&1 || exit 1
  done
done
