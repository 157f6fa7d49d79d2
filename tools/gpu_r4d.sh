#!/bin/bash
# Round 4 profiles for pmc_r04.json: kernel trace + the PMC groups of tools/gpu_profile.sh for the
# headline and every secondary config; then the 2-range compacted probe data point.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash tools/gpu_profile.sh r04_c2c3 --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive --no-secondary || exit 1
for c in c4 c5 lsm lsm_wide many; do
  bash tools/gpu_profile.sh r04_$c --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive || exit 1
done
cd "$ROOT"
for p in 3 2 3 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-inclusive --no-secondary \
      --probe-phases $p >> gpurun_out/r4d_phases.jsonl 2>> gpurun_out/r4d_phases.err || exit 1
done
