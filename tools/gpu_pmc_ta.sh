#!/bin/bash
# Address-path / TLB / L2-queue counters of a bench command, one rocprofv3 --pmc pass per group:
#   tools/gpu_pmc_ta.sh TAG [bench args...]      -> gpurun_out/quick_TAG/{trace,pmc1,pmc2,pmc3}
# (kernel trace first; every pass has its own time limit; stops at the first failure)
set -e
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/quick_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-host-inclusive $*"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-host-inclusive "$@" > "$OUT/trace.log" 2>&1
timeout -k 10 200 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum \
    TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCP_TA_ADDR_STALL_CYCLES_sum \
    TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
    -d "$OUT/pmc1" -o run --output-format csv -- python3 "$ROOT/bench.py" $ARGS > "$OUT/pmc1.log" 2>&1
timeout -k 10 200 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum \
    TCP_TCR_TCP_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum TCC_TAG_STALL_sum TCC_REQ_sum \
    -d "$OUT/pmc2" -o run --output-format csv -- python3 "$ROOT/bench.py" $ARGS > "$OUT/pmc2.log" 2>&1
timeout -k 10 200 rocprofv3 --pmc TA_FLAT_READ_WAVEFRONTS_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_LOAD_WAVEFRONT_sum \
    TD_SPI_STALL_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_REQUEST_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum \
    TCP_TCP_LATENCY_sum SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY \
    -d "$OUT/pmc3" -o run --output-format csv -- python3 "$ROOT/bench.py" $ARGS > "$OUT/pmc3.log" 2>&1
