#!/bin/bash
# k_hash_varlen per key-length shape: one kernel-trace run of tools/varlen_shapes.py per shape,
# stats under gpurun_out/vshape/SHAPE/.  Usage: tools/gpu_varlen_shapes.sh SHAPE...
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for s in "$@"; do
  OUT=$ROOT/gpurun_out/vshape/$s
  mkdir -p "$OUT"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT" -o t --output-format csv -- \
      python3 "$ROOT/tools/varlen_shapes.py" $s > "$OUT/log" 2>&1 || exit 1
done
