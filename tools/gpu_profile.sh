#!/bin/bash
# Profile the bench command on the GPU box: kernel-trace stats, then one PMC pass per counter group
# (never combined with other trace domains).  Usage: tools/gpu_profile.sh TAG [bench args...]
# Writes under gpurun_out/prof_TAG/.  Every GPU step has its own time limit; stops at the first failure.
set -e
TAG=${1:-r01}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS=${@:-"--steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive"}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o bench --output-format csv -- \
    python3 "$ROOT/bench.py" $ARGS > "$OUT/trace.log" 2>&1
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_ATOMIC_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $grp -d "$OUT/pmc$i" -o bench --output-format csv -- \
        python3 "$ROOT/bench.py" $ARGS --steps 3 --warmup 1 > "$OUT/pmc$i.log" 2>&1 || \
        { echo "pmc group '$grp' failed" >> "$OUT/pmc_fail.txt"; tail -5 "$OUT/pmc$i.log" >> "$OUT/pmc_fail.txt"; }
done
