#!/bin/bash
# Build libseb_bloom.so from the product sources of a git revision into tools/ab_lib/NAME/ (CPU,
# here), for an A/B against the in-tree library on the box (SEB_LIB_PATH, tools/gpu_ab_lib.sh).
#   tools/rev_lib.sh NAME [REV]      (REV defaults to HEAD)
set -e
NAME=$1; REV=${2:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/tools/ab_lib/$NAME
SRC=$OUT/src
rm -rf "$SRC" && mkdir -p "$OUT/obj" "$SRC/storage-engines_amd/csrc" "$SRC/include"
(cd "$ROOT" && git archive "$REV" storage-engines_amd/csrc include) | tar -x -C "$SRC"
C=$SRC/storage-engines_amd/csrc
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function"
for f in seb_kernels seb_bucket seb_varlen seb_multiget seb_codec; do
  /opt/rocm/bin/hipcc $FL -c $C/$f.hip -o $OUT/obj/$f.o &
done
/opt/rocm/bin/hipcc $FL -c $C/seb_host.cpp -o $OUT/obj/seb_host.o &
g++ -O2 -std=c++17 -fPIC -ffp-contract=off -c $C/seb_sizing.cpp -o $OUT/obj/seb_sizing.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libseb_bloom.so $OUT/obj/*.o -Wl,-rpath,/opt/rocm/lib
echo "$OUT/libseb_bloom.so"
