#!/bin/bash
# Round 5: settle scatter_tiles_exact: the parity subset with the option in
# every scatter test (bins x {tiles_exact 0, 1}), then an alternating A/B of the headline.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "key_sources or scatter_bins" > gpurun_out/r5a_tests.log 2>&1 || { tail -30 gpurun_out/r5a_tests.log; exit 1; }
tail -1 gpurun_out/r5a_tests.log
bash tools/gpu_ab_env.sh tiles "SEB_SCATTER_TILES_EXACT=1" "SEB_SCATTER_TILES_EXACT=0"
