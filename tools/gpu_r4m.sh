#!/bin/bash
# Round 4 (session 2): the pruned pipelined bin scatter (48/32 slots, runs padded to 8), apply
# skipping the padding; A/B against apply OR-ing the padding and against the counting sort.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "scatter_bins or fresh_build or c2_c3_10m or bucketed or c4_varlen_device or caller_workspace" \
    > gpurun_out/r4m_tests.log 2>&1 || { tail -30 gpurun_out/r4m_tests.log; exit 1; }
tail -2 gpurun_out/r4m_tests.log
bash tools/gpu_ab_env.sh pruned "SEB_SCATTER_BINS=1" "SEB_LIB_PATH=$ROOT/tools/ab_lib/orpad/libseb_bloom.so" "SEB_SCATTER_BINS=0"
