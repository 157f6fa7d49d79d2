#!/bin/bash
# Round 5: 4-rank gloo rehearsal at HEAD (per-rank records), then the lsm / lsm_wide re-profile
# after the chunked unpermute.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash tools/gpu_rehearse.sh 4 > gpurun_out/r5j_rehearse4.txt 2>&1 || { tail -30 gpurun_out/r5j_rehearse4.txt; exit 1; }
cat gpurun_out/r5j_rehearse4.txt | grep -v "^   rank" | head -30
bash tools/gpu_r5_prof.sh lsm lsm_wide
