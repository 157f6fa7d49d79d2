#!/bin/bash
# The all-gather batch path (--batch-origin spread) on the one GPU: the multi-rank GPU tests, then
# the 4-rank gloo rehearsal of c2c3 with its root_broadcast and resident_batch secondaries
# (parity only; gloo times mean nothing).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=gpurun_out/${TAG:-r5p}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_multirank.py \
    > $OUT/multirank.log 2>&1 || { tail -40 $OUT/multirank.log; exit 1; }
tail -1 $OUT/multirank.log
timeout -k 10 300 python bench.py --gpus 4 --dist-backend gloo --steps 4 --warmup 2 --no-cpu-baseline \
    --no-host-inclusive > $OUT/c2c3_4.json 2> $OUT/c2c3_4.err || { tail -20 $OUT/c2c3_4.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/c2c3_4.json').read().strip().splitlines()[-1])
print(d['n_gpus'], d['devices'], d['parity'], d['config']['parallelism'])
print('root_broadcast', d['root_broadcast']['parity'], 'resident', d['resident_batch']['parity'])
for r in d['per_rank']: print(r['rank'], r['kernel_ms'], r['wait_ms'])
"
