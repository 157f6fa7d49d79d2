#!/bin/bash
# Re-profile at HEAD: kernel trace + PMC passes per config, through
# tools/gpu_profile.sh.  Usage: tools/gpu_reprofile.sh CONFIG... (c2c3 c4 c5 lsm lsm_wide)
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
for cfg in "$@"; do
  bash tools/gpu_profile.sh ${PREFIX:-r05}_$cfg --config $cfg --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive \
      --no-secondary || exit 1
done
