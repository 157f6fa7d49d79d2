#!/bin/bash
# Round 4 (session 2): fixed-bin scatter variants (runs padded to 8 or 2, split count/fill arrays)
# against the counting sort: parity, then a three-way A/B of the default step.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "scatter_bins or fresh_build or c2_c3_10m or bucketed or caller_workspace" \
    > gpurun_out/r4j_tests.log 2>&1 || { tail -30 gpurun_out/r4j_tests.log; exit 1; }
tail -3 gpurun_out/r4j_tests.log
bash tools/gpu_ab_env.sh bins2 "SEB_SCATTER_BINS=1" "SEB_SCATTER_BINS=2" "SEB_SCATTER_BINS=0"
