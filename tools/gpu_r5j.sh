#!/bin/bash
# Round 5: 4-rank gloo rehearsal at HEAD (per-rank records), then the lsm / lsm_wide re-profile
# after the chunked unpermute.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "registry or lsm or multiget" > gpurun_out/r5j_tests.log 2>&1 || { tail -40 gpurun_out/r5j_tests.log; exit 1; }
tail -1 gpurun_out/r5j_tests.log
bash tools/gpu_rehearse.sh 4 > gpurun_out/r5j_rehearse4.txt 2>&1 || { tail -30 gpurun_out/r5j_rehearse4.txt; exit 1; }
cat gpurun_out/r5j_rehearse4.txt | grep -v "^   rank" | head -30
bash tools/gpu_r5_prof.sh lsm lsm_wide
