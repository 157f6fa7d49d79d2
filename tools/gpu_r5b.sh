#!/bin/bash
# Round 5: (1) parity of the scatter_tiles_exact option, of the MultiGet's new ordering (stable
# chunk ranks, answers in sorted rows + unpermute) and of the C4 long-key pass (varlen_long);
# (2) A/B of the MultiGet against the round-4 library (tools/ab_lib/mg_old) on lsm / lsm_wide.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out/r5b
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "key_sources or scatter_bins or registry or lsm or multiget or varlen or c4" > gpurun_out/r5b/tests.log 2>&1 \
    || { tail -40 gpurun_out/r5b/tests.log; exit 1; }
tail -1 gpurun_out/r5b/tests.log
for cfg in lsm lsm_wide; do
  for r in 1 2; do
    timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 > gpurun_out/r5b/new_$cfg.$r.json 2>gpurun_out/r5b/err || exit 1
    SEB_LIB_PATH=$ROOT/tools/ab_lib/mg_old/libseb_bloom.so timeout -k 10 200 python bench.py --config $cfg --steps 20 \
        --warmup 3 > gpurun_out/r5b/old_$cfg.$r.json 2>gpurun_out/r5b/err || exit 1
  done
done
python3 - <<'PY'
import json, glob, os
for f in sorted(glob.glob("gpurun_out/r5b/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f"{os.path.basename(f):22s} {d['value']:9.1f} ms {d['ms_per_step']} {d['parity'][:9]}")
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/r5b/prof_lsm" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" --config lsm --steps 10 --warmup 3 > "$ROOT/gpurun_out/r5b/prof_lsm.log" 2>&1 || exit 1
cd "$ROOT"
