#!/bin/bash
# Round 5 re-profile (part 1): c2c3 and c4 at HEAD, and c4 with the long-key pass on builds
# (SEB_VARLEN_LONG=1) for its VALU counts.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash tools/gpu_r5_prof.sh c2c3 c4 || exit 1
SEB_VARLEN_LONG=1 bash tools/gpu_profile.sh r05_c4_long1 --config c4 --steps 10 --warmup 3 --no-cpu-baseline \
    --no-host-inclusive --no-secondary
