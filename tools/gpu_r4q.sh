#!/bin/bash
# Round 4 final profiles (session 2, after the bin scatter): kernel trace + PMC of c2c3 and C4.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash tools/gpu_profile.sh r04g_c2c3 --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive --no-secondary || exit 1
bash tools/gpu_profile.sh r04g_c4 --config c4 --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive || exit 1
