#!/bin/bash
# Round 5: the C4 long-key pass with batched loads: parity (varlen tests), then A/B of
# varlen_long 0 (off) / 1 (builds only) / 2 (builds and the fused probe) on --config c4.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out/r5f
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "varlen or c4" > gpurun_out/r5f/tests.log 2>&1 || { tail -40 gpurun_out/r5f/tests.log; exit 1; }
tail -1 gpurun_out/r5f/tests.log
bash tools/gpu_ab_env.sh ${TAG:-vlong2} "SEB_VARLEN_LONG=0" "SEB_VARLEN_LONG=1" "SEB_VARLEN_LONG=2" -- --config c4
