#!/bin/bash
# C4 with the build of step j+1 overlapped with the probe of step j (--overlap 1) against the
# default, alternating on one box; kernel traces of both.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=gpurun_out/${TAG:-r5r}
mkdir -p $OUT
for rep in 1 2; do
  for ov in 0 1; do
    timeout -k 10 120 python bench.py --config c4 --steps 20 --warmup 3 --no-cpu-baseline --overlap $ov \
        > $OUT/c4_ov$ov.$rep.json 2> $OUT/c4_ov$ov.$rep.err || { tail -20 $OUT/c4_ov$ov.$rep.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], d['ms_per_step'], d.get('build_ms'), d.get('probe_ms'), d['parity'][:30])" $OUT/c4_ov$ov.$rep.json
  done
done
cd /tmp && export TMPDIR=/tmp
for ov in 0 1; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof_ov$ov -o run -- python3 $ROOT/bench.py --config c4 \
      --steps 10 --warmup 3 --no-cpu-baseline --overlap $ov > $ROOT/$OUT/prof_ov$ov.log 2>&1 || exit 1
done
