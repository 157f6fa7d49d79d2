#!/bin/bash
# Round 4 (session 2): 32-slot bins (4 write-out lanes per bucket; ~6% of bucket-rounds past the bin)
# against 48-slot bins for C2.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "scatter_bins or c2_c3_10m" > gpurun_out/r4aa_tests.log 2>&1 || { tail -30 gpurun_out/r4aa_tests.log; exit 1; }
tail -1 gpurun_out/r4aa_tests.log
bash tools/gpu_ab_env.sh s32 "SEB_SCATTER_BINS=1" "SEB_SCATTER_BINS=2"
