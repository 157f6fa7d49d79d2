#!/bin/bash
# Round 5: A/B of scatter_tiles_exact on the headline and of the C4 long-key pass (varlen_long).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash tools/gpu_ab_env.sh vlong "SEB_VARLEN_LONG=1" "SEB_VARLEN_LONG=0" -- --config c4 || exit 1
bash tools/gpu_ab_env.sh tiles "SEB_SCATTER_TILES_EXACT=1" "SEB_SCATTER_TILES_EXACT=0"
