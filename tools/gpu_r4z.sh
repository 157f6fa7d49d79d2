#!/bin/bash
# Round 4 (session 2): phase 0 hashing with no branch around it (clamped index) vs the branch.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "probe_paths or phased_probe_small or c2_c3_10m or packed" > gpurun_out/r4z_tests.log 2>&1 || { tail -30 gpurun_out/r4z_tests.log; exit 1; }
tail -1 gpurun_out/r4z_tests.log
bash tools/gpu_ab_env.sh c0br "SEB_SCATTER_BINS=1" "SEB_LIB_PATH=$ROOT/tools/ab_lib/c0br/libseb_bloom.so"
