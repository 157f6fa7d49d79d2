#!/bin/bash
# Quick kernel-trace + one SQ counter pass of a bench command: tools/gpu_pmc_quick.sh TAG [bench args...]
# Writes gpurun_out/quick_TAG/{trace,pmc}.  Each GPU step has its own time limit.
set -e
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/quick_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-host-inclusive "$@" > "$OUT/trace.log" 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
    -d "$OUT/pmc" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-host-inclusive "$@" > "$OUT/pmc.log" 2>&1
