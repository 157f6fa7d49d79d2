#!/bin/bash
# Round 5: parity of the final MultiGet ordering, then A/B of the C4 long-key pass (varlen_long)
# and of scatter_tiles_exact on the headline.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out/r5c
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "registry or lsm or multiget" > gpurun_out/r5c/tests.log 2>&1 || { tail -40 gpurun_out/r5c/tests.log; exit 1; }
tail -1 gpurun_out/r5c/tests.log
bash tools/gpu_ab_env.sh vlong "SEB_VARLEN_LONG=1" "SEB_VARLEN_LONG=0" -- --config c4 || exit 1
bash tools/gpu_ab_env.sh tiles "SEB_SCATTER_TILES_EXACT=1" "SEB_SCATTER_TILES_EXACT=0"
