#!/bin/bash
# Kernel stats of one bench command: tools/quick_stats.sh TAG [bench args...] -> gpurun_out/qs_TAG/
set -e
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/qs_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-host-inclusive --no-secondary "$@" \
    > "$OUT/bench.json" 2> "$OUT/bench.err"
f=$(find "$OUT/trace" -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f'{r["Name"][:90]:90s} {int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:9.1f} us')
PY
