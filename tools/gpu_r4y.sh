#!/bin/bash
# Round 4 (session 2): the bin scatter's pipeline written for G keys per step (G = 1) against the
# plain single-key form (tools/diag/scatter_pipeline_single_key.patch), same box.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash tools/gpu_ab_env.sh gform "SEB_SCATTER_BINS=1" "SEB_LIB_PATH=$ROOT/tools/ab_lib/simple/libseb_bloom.so"
