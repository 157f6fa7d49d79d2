#!/bin/bash
# Kernel-trace stats of the bench with the in-tree library and with SEB_LIB_PATH=ALT_LIB:
# tools/gpu_ab_prof.sh TAG ALT_LIB [bench args...]  -> gpurun_out/abprof_TAG/{new,old}/
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; ALT=$2; shift 2
OUT=$ROOT/gpurun_out/abprof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/new" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-host-inclusive "$@" > "$OUT/new.log" 2>&1 || exit 1
export SEB_LIB_PATH=$ROOT/$ALT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/old" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-host-inclusive "$@" > "$OUT/old.log" 2>&1
