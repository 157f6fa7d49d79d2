#!/bin/bash
# Round 4 (session 2): phase 0 of the compacted probe as a grid-stride loop with the next key
# prefetched (probe_c0_grid workgroups) against one key per thread.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "probe_paths or phased_probe_small or c2_c3_10m" > gpurun_out/r4o_tests.log 2>&1 || { tail -30 gpurun_out/r4o_tests.log; exit 1; }
tail -2 gpurun_out/r4o_tests.log
bash tools/gpu_ab_env.sh c0grid "SEB_PROBE_C0_GRID=0" "SEB_PROBE_C0_GRID=1024" "SEB_PROBE_C0_GRID=2048" "SEB_PROBE_C0_GRID=4096" "SEB_PROBE_C0_GRID=8192"
