#!/bin/bash
# One PMC pass per counter group for the bench under each option setting:
#   tools/gpu_pmc_env.sh TAG "ENV_A" ["ENV_B" ...] -- [bench args]
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
V=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do V+=("$1"); shift; done
[ "$1" = "--" ] && shift
OUT=$ROOT/gpurun_out/pmcenv_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
G=("SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES"
   "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY")
for i in "${!V[@]}"; do
  for g in "${!G[@]}"; do
    env ${V[$i]} timeout -s KILL 90 rocprofv3 --pmc ${G[$g]} -d "$OUT/v$i.g$g" -o run --output-format csv -- \
        python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-host-inclusive --no-secondary "$@" \
        > "$OUT/v$i.g$g.log" 2>&1 || { echo "v$i g$g failed" >> "$OUT/fail.txt"; tail -3 "$OUT/v$i.g$g.log" >> "$OUT/fail.txt"; }
  done
done
exit 0
