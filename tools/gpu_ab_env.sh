#!/bin/bash
# A/B/... of option settings or library builds on one box:
#   tools/gpu_ab_env.sh TAG "ENV_A" "ENV_B" [...] -- [bench args...]
# e.g. tools/gpu_ab_env.sh bins "SEB_SCATTER_BINS=1" "SEB_SCATTER_BINS=0" "SEB_LIB_PATH=$PWD/tools/ab_lib/x/libseb_bloom.so"
# (an ENV may hold several VAR=VAL separated by spaces).  Alternates three bench runs per variant,
# then one kernel trace per variant; prints value / build_ms / probe_ms per run.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
V=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do V+=("$1"); shift; done
[ "$1" = "--" ] && shift
OUT=$ROOT/gpurun_out/abenv_$TAG
mkdir -p "$OUT"
for r in 1 2 3; do
  for i in "${!V[@]}"; do
    env ${V[$i]} timeout -k 10 200 python "$ROOT/bench.py" --steps 30 --warmup 5 --no-cpu-baseline --no-host-inclusive \
        --no-secondary "$@" > "$OUT/v$i.$r.json" 2> "$OUT/v$i.$r.err" || exit 1
  done
done
for i in "${!V[@]}"; do echo "v$i: ${V[$i]}"; done
python3 - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "v*.json"))):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f"{os.path.basename(f):12s} {d['value']:9.1f} {d.get('build_ms')} {d.get('probe_ms')} {d['parity'][:9]}")
PY
cd /tmp && export TMPDIR=/tmp
for i in "${!V[@]}"; do
  env ${V[$i]} timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof_v$i" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-host-inclusive --no-secondary "$@" \
      > "$OUT/prof_v$i.log" 2>&1 || exit 1
done
