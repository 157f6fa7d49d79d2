#!/bin/bash
# A/B of libseb_bloom.so builds on the MultiGet configs (GPU box): kernel-trace stats of
# bench.py --config lsm and lsm_wide per build.  Usage: bash tools/mg_ab.sh TAG NAME... (NAME = a
# tools/ab_lib/NAME build, or "product")
set -e
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for name in "$@"; do
  lib=$ROOT/tools/ab_lib/$name/libseb_bloom.so
  [ "$name" = product ] && lib=$ROOT/storage-engines_amd/lib/libseb_bloom.so
  for c in lsm lsm_wide; do
    mkdir -p "$ROOT/gpurun_out/$TAG/$name"
    SEB_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/$TAG/$name/$c" -o k \
      --output-format csv -- python3 "$ROOT/bench.py" --config $c --steps 10 --warmup 3 --no-cpu-baseline \
      > "$ROOT/gpurun_out/$TAG/$name/$c.json" 2> "$ROOT/gpurun_out/$TAG/$name/$c.err"
  done
done
