#!/bin/bash
# Round 4 (session 2): phase 0 positions from the packed word (one residue/flag computation),
# new key-source tests for the bin scatter; A/B against computing them twice.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "key_sources or scatter_bins or probe_paths or phased_probe_small or packed or emit or c2_c3_10m or sliced" \
    > gpurun_out/r4v_tests.log 2>&1 || { tail -30 gpurun_out/r4v_tests.log; exit 1; }
tail -2 gpurun_out/r4v_tests.log
bash tools/gpu_ab_env.sh once "SEB_SCATTER_BINS=1" "SEB_LIB_PATH=$ROOT/tools/ab_lib/twice/libseb_bloom.so"
