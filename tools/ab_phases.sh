#!/bin/bash
# Phase counts of the phased probe, compacted (1) and not (0): c2c3 bench lines -> gpurun_out/abp/
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/abp
mkdir -p "$OUT"
ARGS="--steps 30 --warmup 5 --no-cpu-baseline --no-host-inclusive --no-secondary"
for p in ${PHASES:-3 4 5 6}; do
  for c in ${COMPACT:-1}; do
    timeout -k 10 120 python3 "$ROOT/bench.py" $ARGS --probe-compact $c --probe-phases $p > "$OUT/p${p}_c${c}.json"
  done
done
python3 - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(os.path.basename(f), d["value"], d["build_ms"], d["probe_ms"], d["parity"][:9])
PY
