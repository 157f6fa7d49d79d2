#!/bin/bash
# Round 4 (session 2): the fixed-bin scatter.  Parity of both scatters, then an A/B of the default step.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "scatter_bins or fresh_build or c2_c3_10m or bucketed or c4_varlen_device or caller_workspace" \
    > gpurun_out/r4i_tests.log 2>&1 || { tail -30 gpurun_out/r4i_tests.log; exit 1; }
tail -3 gpurun_out/r4i_tests.log
bash tools/gpu_ab_env.sh bins "SEB_SCATTER_BINS=1" "SEB_SCATTER_BINS=0"
