#!/bin/bash
# A/B of library variants built by tools/diag_lib.sh (tools/ab_lib/NAME/libseb_bloom.so; "head" =
# a copy of the in-tree library): alternating bench runs of CFGS for every variant (REPS rounds),
# then a kernel trace of each variant on PCFGS.  Parity: every bench line checks its golden digest.
#   TAG=x VARIANTS="head bt512" CFGS="lsm lsm_wide" PCFGS="lsm" bash tools/gpu_ab_variants.sh
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=gpurun_out/${TAG:-abv}
mkdir -p $OUT
for r in $(seq 1 ${REPS:-2}); do
  for cfg in ${CFGS:-lsm}; do
    for v in ${VARIANTS:-head}; do
      SEB_LIB_PATH=$ROOT/tools/ab_lib/$v/libseb_bloom.so timeout -k 10 200 python bench.py --config $cfg --steps 20 \
          --warmup 3 --no-cpu-baseline > $OUT/${v}_$cfg.$r.json 2>$OUT/err || { tail -20 $OUT/err; exit 1; }
    done
  done
done
OUT=$OUT python3 - <<'PY'
import json, glob, os
for f in sorted(glob.glob(os.environ["OUT"] + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f"{os.path.basename(f):26s} {d['value']:9.1f} ms {d['ms_per_step']} {d.get('build_ms')} {d.get('probe_ms')} {d['parity'][:9]}")
PY
cd /tmp && export TMPDIR=/tmp
for cfg in ${PCFGS:-}; do
  for v in ${VARIANTS:-head}; do
    SEB_LIB_PATH=$ROOT/tools/ab_lib/$v/libseb_bloom.so timeout -k 10 200 rocprofv3 --kernel-trace --stats \
        -d "$ROOT/$OUT/prof_${v}_$cfg" -o run --output-format csv -- python3 "$ROOT/bench.py" --config $cfg --steps 10 \
        --warmup 3 --no-cpu-baseline > "$ROOT/$OUT/prof_${v}_$cfg.log" 2>&1 || exit 1
    python3 - "$ROOT/$OUT/prof_${v}_$cfg/run_kernel_stats.csv" "$v $cfg" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print("  ", sys.argv[2], "  ".join(f"{r['Name'].split('(')[0].split('::')[-1][:22]} {float(r['AverageNs'])/1e3:.1f}"
                               for r in rows if "seb::" in r["Name"])[:400])
PY
  done
done
