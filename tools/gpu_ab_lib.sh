#!/bin/bash
# A/B of two library builds on one box: tools/gpu_ab_lib.sh TAG ALT_LIB [bench args...]
# Runs the bench with the in-tree library and with SEB_LIB_PATH=ALT_LIB, alternating, three times
# each, and prints value / build_ms / probe_ms per run.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; ALT=$2; shift 2
OUT=$ROOT/gpurun_out/ab_$TAG
mkdir -p "$OUT"
for r in 1 2 3; do
  timeout -k 10 200 python "$ROOT/bench.py" --steps 30 --warmup 5 --no-cpu-baseline --no-host-inclusive \
      --no-secondary "$@" > "$OUT/new$r.json" 2> "$OUT/new$r.err" || exit 1
  SEB_LIB_PATH=$ROOT/$ALT timeout -k 10 200 python "$ROOT/bench.py" --steps 30 --warmup 5 --no-cpu-baseline \
      --no-host-inclusive --no-secondary "$@" > "$OUT/old$r.json" 2> "$OUT/old$r.err" || exit 1
done
python3 - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f"{os.path.basename(f):12s} {d['value']:9.1f} {d.get('build_ms')} {d.get('probe_ms')} {d['parity'][:9]}")
PY
