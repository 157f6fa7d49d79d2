#!/bin/bash
# r4f (SDWA parity + A/B) then r4e (GPU suite, smoke, default bench, 4-rank rehearsal) in one call.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
bash "$ROOT/tools/gpu_r4f.sh" || exit 1
bash "$ROOT/tools/gpu_r4e.sh" || exit 1
