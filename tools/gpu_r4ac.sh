#!/bin/bash
# Round 4 (session 2): bin scatter rounds shrunk so the tiles fill all 256 CUs (256 tiles of 8
# rounds of 4883 keys for C2 instead of 245 of 8 x 5120).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
export SEB_SCATTER_TILES_EXACT=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "key_sources or scatter_bins or fresh_build or c2_c3_10m or c4_varlen or bucketed" \
    > gpurun_out/r4ac_tests.log 2>&1 || { tail -30 gpurun_out/r4ac_tests.log; exit 1; }
tail -1 gpurun_out/r4ac_tests.log
unset SEB_SCATTER_TILES_EXACT
bash tools/gpu_ab_env.sh tiles "SEB_SCATTER_TILES_EXACT=1" "SEB_SCATTER_TILES_EXACT=0"
