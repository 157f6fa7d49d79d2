#!/bin/bash
# Round 4 final profiles (after the SDWA change): kernel trace + PMC of the default c2c3 step and of C4.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash tools/gpu_profile.sh r04f_c2c3 --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive --no-secondary || exit 1
bash tools/gpu_profile.sh r04f_c4 --config c4 --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive || exit 1
bash tools/gpu_profile.sh r04f_c5 --config c5 --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive || exit 1
