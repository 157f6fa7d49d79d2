#!/bin/bash
# Round 4 (session 2): bin scatter write-out one lane per bucket (scatter_bins 2) vs 6 lanes per bucket.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "scatter_bins or c2_c3_10m" > gpurun_out/r4s_tests.log 2>&1 || { tail -30 gpurun_out/r4s_tests.log; exit 1; }
tail -2 gpurun_out/r4s_tests.log
bash tools/gpu_ab_env.sh lpb "SEB_SCATTER_BINS=1" "SEB_SCATTER_BINS=2"
