#!/bin/bash
# A/B of bench option sets on c2c3: VARIANTS="name:--opt a --opt2 b;name2:..." tools/ab_opts.sh TAG
# Each variant runs twice, alternating; lines in gpurun_out/abo_TAG/.
set -e
TAG=$1
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/abo_$TAG
mkdir -p "$OUT"
ARGS="--steps 30 --warmup 5 --no-cpu-baseline --no-host-inclusive --no-secondary ${EXTRA:-}"
IFS=';' read -ra VS <<< "$VARIANTS"
for r in 1 2; do
  for v in "${VS[@]}"; do
    name=${v%%:*}; opts=${v#*:}
    timeout -k 10 120 python3 "$ROOT/bench.py" $ARGS $opts > "$OUT/${name}_$r.json"
  done
done
python3 - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f"{os.path.basename(f):24s} {d['value']:9.1f} {d.get('build_ms')} {d.get('probe_ms')} {d['parity'][:9]}")
PY
