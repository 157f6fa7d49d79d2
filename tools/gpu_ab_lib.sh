#!/bin/bash
# A/B of two library builds on one box: tools/gpu_ab_lib.sh TAG ALT_LIB [bench args...]
# Runs the bench with the in-tree library and with SEB_LIB_PATH=ALT_LIB, alternating, twice each.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; ALT=$2; shift 2
OUT=$ROOT/gpurun_out/ab_$TAG
mkdir -p "$OUT"
for r in 1 2; do
  timeout -k 10 200 python "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive "$@" \
      > "$OUT/new$r.json" 2> "$OUT/new$r.err" || exit 1
  SEB_LIB_PATH=$ROOT/$ALT timeout -k 10 200 python "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline \
      --no-host-inclusive "$@" > "$OUT/old$r.json" 2> "$OUT/old$r.err" || exit 1
done
