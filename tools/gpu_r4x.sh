#!/bin/bash
# Round 4 (session 2): parity of the build paths after the pipeline cleanup, one bench line.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out/r4x
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "key_sources or scatter_bins or fresh_build or c2_c3_10m or c4_varlen or bucketed or caller_workspace" \
    > gpurun_out/r4x/tests.log 2>&1 || { tail -30 gpurun_out/r4x/tests.log; exit 1; }
tail -1 gpurun_out/r4x/tests.log
timeout -k 10 300 python bench.py --no-secondary --no-cpu-baseline --no-host-inclusive > gpurun_out/r4x/bench.json 2> gpurun_out/r4x/bench.err || exit 1
tail -c 400 gpurun_out/r4x/bench.json
