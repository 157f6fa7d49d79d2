#!/bin/bash
# Overlap experiment: bench c2c3 with/without --overlap (build j+1 on its own stream beside probe j)
# for the in-tree library and the diagnostic builds given as arguments (tools/ab_lib/NAME).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/ov
mkdir -p "$OUT"
for lib in default "$@"; do
  for ov in 0 1; do
    for kpt in 5 4; do
      if [ "$lib" = default ]; then L=""; else L="$ROOT/tools/ab_lib/$lib/libseb_bloom.so"; fi
      SEB_LIB_PATH=$L timeout -k 10 120 python "$ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline \
          --no-host-inclusive --overlap $ov --scatter-kpt $kpt > "$OUT/${lib}_ov${ov}_k${kpt}.json" 2> "$OUT/${lib}_ov${ov}_k${kpt}.err" || exit 1
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['build_ms'], d['probe_ms'], d['parity'][:9])" \
          "$OUT/${lib}_ov${ov}_k${kpt}.json" "${lib}_ov${ov}_k${kpt}"
    done
  done
done
