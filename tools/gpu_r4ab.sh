#!/bin/bash
# Round 4 (session 2): apply with 4 chunk loads in flight per thread (issued before the counts are
# consulted) against one (tools/diag/apply_one_load_in_flight.patch); c2c3 and C4.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "key_sources or scatter_bins or fresh_build or c2_c3_10m or c4_varlen or bucketed or caller_workspace" \
    > gpurun_out/r4ab_tests.log 2>&1 || { tail -30 gpurun_out/r4ab_tests.log; exit 1; }
tail -1 gpurun_out/r4ab_tests.log
bash tools/gpu_ab_env.sh u4 "SEB_SCATTER_BINS=1" "SEB_LIB_PATH=$ROOT/tools/ab_lib/onel/libseb_bloom.so"
