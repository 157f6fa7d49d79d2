#!/bin/bash
# Kernel-trace stats per bench variant: tools/gpu_prof_variants.sh TAG "name=bench flags" ...
# -> gpurun_out/pv_TAG/NAME/ ; summarise with tools/pv_table.py TAG
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  name=${v%%=*}; flags=${v#*=}
  OUT=$ROOT/gpurun_out/pv_$TAG/$name
  mkdir -p "$OUT"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-host-inclusive $flags > "$OUT/log" 2>&1 || exit 1
done
