#!/bin/bash
# Multi-rank rehearsal on the one-GPU box: N ranks (default 4), all on cuda:0, gloo instead of
# RCCL (RCCL refuses two ranks on one device).  Checks the N > 1 code paths (broadcast pipeline,
# all-gather pipeline, sharded filters, mask-plane gather, the key x filter grid, sharded build, partitioned probe) for parity; the times mean
# nothing.  Usage: tools/gpu_rehearse.sh [N].  Writes gpurun_out/rehearse_N_<config>.json.
set -e
N=${1:-4}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
port=29611
for cfg in "c2c3" "c2c3 --batch-origin root" "c2c3 --bcast keys" "c5" "c5_2d" "c5_2d --c5-groups 2" "c2_sharded" "c3_partitioned"; do
    tag=$(echo "$cfg" | tr ' ' '_' | tr -d '-')
    port=$((port + 1))
    timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
        --master-port $port "$ROOT/bench.py" --gpus "$N" --steps 4 --warmup 2 --dist-backend gloo \
        --no-cpu-baseline --no-host-inclusive --config $cfg > "$OUT/rehearse_${N}_${tag}.json" 2> "$OUT/rehearse_${N}_${tag}.err"
    python3 -c "
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d['n_gpus'], d['parity'], d.get('root_broadcast', {}).get('parity', ''),
      d.get('resident_batch', {}).get('parity', ''))
print('   devices', d['devices'], 'rank_check', d['rank_check'])
for r in d['per_rank']:
    print('   rank', r['rank'], r['device']['pci'], r['backend'], 'world', r['world_size'], 'ones', r['allreduce_ones'],
          'kernel_ms', r['kernel_ms'], 'wait_ms', r['wait_ms'], 'elapsed_s', r['elapsed_s'])
" "$OUT/rehearse_${N}_${tag}.json" "$cfg"
done
