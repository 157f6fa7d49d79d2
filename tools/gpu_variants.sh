#!/bin/bash
# A/B bench variants: each arg is "name=bench flags" (one JSON line each) under gpurun_out/variants_TAG/.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/variants_$1
mkdir -p "$OUT"
shift
for v in "$@"; do
  name=${v%%=*}; flags=${v#*=}
  timeout -k 10 200 python "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive $flags \
      > "$OUT/$name.json" 2> "$OUT/$name.err" || exit 1
done
