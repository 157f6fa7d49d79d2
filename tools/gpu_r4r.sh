#!/bin/bash
# Round 4 (session 2): apply loading the regions' first 16 chunks before the counts, A/B against
# loading them after (tools/diag/apply_no_head_loads.patch).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "scatter_bins or fresh_build or c2_c3_10m or bucketed or c4_varlen_device" > gpurun_out/r4r_tests.log 2>&1 || { tail -30 gpurun_out/r4r_tests.log; exit 1; }
tail -2 gpurun_out/r4r_tests.log
bash tools/gpu_ab_env.sh head "SEB_SCATTER_BINS=1" "SEB_LIB_PATH=$ROOT/tools/ab_lib/nohead/libseb_bloom.so"
