#!/bin/bash
# Round 4 (session 2): fixed-bin scatter variants (deferred bin overflow, pad 8 / pad 2 / pad 2 with
# 4 keys per thread) against the counting sort: parity, A/B, PMC.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "scatter_bins or fresh_build or c2_c3_10m" > gpurun_out/r4k_tests.log 2>&1 || { tail -30 gpurun_out/r4k_tests.log; exit 1; }
tail -2 gpurun_out/r4k_tests.log
bash tools/gpu_ab_env.sh bins3 "SEB_SCATTER_BINS=4" "SEB_SCATTER_BINS=5" "SEB_SCATTER_BINS=2" "SEB_SCATTER_BINS=0" || exit 1
bash tools/gpu_pmc_env.sh bins3 "SEB_SCATTER_BINS=4" "SEB_SCATTER_BINS=0"
