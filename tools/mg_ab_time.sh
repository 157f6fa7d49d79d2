#!/bin/bash
# MultiGet library A/B by the bench's own clock (no profiler): bench.py --config lsm / lsm_wide at
# the default 50 warm-up + 100 timed steps, libraries alternating, ROUNDS rounds.
# Usage (GPU box): bash tools/mg_ab_time.sh TAG ROUNDS NAME...  (NAME = tools/ab_lib/NAME or "product")
set -e
TAG=$1; ROUNDS=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for name in "$@"; do
    lib=$ROOT/tools/ab_lib/$name/libseb_bloom.so
    [ "$name" = product ] && lib=$ROOT/storage-engines_amd/lib/libseb_bloom.so
    for c in lsm lsm_wide; do
      SEB_LIB_PATH=$lib timeout -k 10 200 python3 "$ROOT/bench.py" --config $c --no-cpu-baseline \
        > "$OUT/$name.$c.$r.json" 2> "$OUT/$name.$c.$r.err"
    done
  done
done
python3 - "$OUT" <<'PY'
import glob, json, os, sys
rows = {}
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    name, cfg, r, _ = os.path.basename(f).split(".")
    d = json.loads(open(f).read().strip().splitlines()[-1])
    rows.setdefault((name, cfg), []).append((d["ms_per_step"], d["parity"][:9]))
for (name, cfg), v in sorted(rows.items()):
    print(f"{name:12s} {cfg:9s}", " ".join(f"{ms:.4f}" for ms, _ in v), {p for _, p in v})
PY
