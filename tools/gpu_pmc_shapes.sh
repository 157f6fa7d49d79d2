#!/bin/bash
# Kernel trace + one SQ counter pass of tools/varlen_shapes.py per shape, laid out like
# tools/gpu_pmc_quick.sh (gpurun_out/quick_vs_SHAPE/{trace,pmc}) for tools/pmc_table.py.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for s in "$@"; do
  OUT=$ROOT/gpurun_out/quick_vs_$s
  mkdir -p "$OUT"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
      python3 "$ROOT/tools/varlen_shapes.py" $s > "$OUT/trace.log" 2>&1
  timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
      -d "$OUT/pmc" -o run --output-format csv -- python3 "$ROOT/tools/varlen_shapes.py" $s > "$OUT/pmc.log" 2>&1
done
