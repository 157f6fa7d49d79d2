#!/bin/bash
# Round 4 (session 2): pipelined fixed-bin scatter, write-out in 6-lane bucket groups; 5 or 6 keys
# per thread, runs padded to 8 or 2; apply walking to the longest region (A/B against the cap walk).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "scatter_bins or fresh_build or c2_c3_10m" > gpurun_out/r4l_tests.log 2>&1 || { tail -30 gpurun_out/r4l_tests.log; exit 1; }
tail -2 gpurun_out/r4l_tests.log
bash tools/gpu_ab_env.sh pipe "SEB_SCATTER_BINS=4" "SEB_SCATTER_BINS=5" "SEB_SCATTER_BINS=6" "SEB_SCATTER_BINS=7" \
    "SEB_SCATTER_BINS=0" "SEB_SCATTER_BINS=0 SEB_LIB_PATH=$ROOT/tools/ab_lib/apply_cap/libseb_bloom.so"
