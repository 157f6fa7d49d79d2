#!/bin/bash
# A/B of the compacted phased probe (probe_compact 1) against every word through every phase (0):
# the c2c3 bench, alternating, two pairs.  Writes gpurun_out/abc/*.json.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/abc
mkdir -p "$OUT"
ARGS="--steps 30 --warmup 5 --no-cpu-baseline --no-host-inclusive --no-secondary"
for r in 1 2; do
  for c in 1 0; do
    timeout -k 10 120 python3 "$ROOT/bench.py" $ARGS --probe-compact $c > "$OUT/c${c}_$r.json"
  done
done
python3 - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(os.path.basename(f), d["value"], d["build_ms"], d["probe_ms"], d["parity"][:9])
PY
