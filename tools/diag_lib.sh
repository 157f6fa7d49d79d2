#!/bin/bash
# Build a diagnostic variant of libseb_bloom.so with extra -D flags into tools/ab_lib/NAME/ (CPU,
# here): tools/diag_lib.sh NAME -DSEB_DIAG_...   Run it on the box with SEB_LIB_PATH=tools/ab_lib/NAME/libseb_bloom.so.
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/tools/ab_lib/$NAME
mkdir -p "$OUT/obj"
C=$ROOT/storage-engines_amd/csrc
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function $*"
for f in seb_kernels seb_bucket seb_varlen seb_multiget seb_codec; do
  /opt/rocm/bin/hipcc $FL -c $C/$f.hip -o $OUT/obj/$f.o &
done
/opt/rocm/bin/hipcc $FL -c $C/seb_host.cpp -o $OUT/obj/seb_host.o &
g++ -O2 -std=c++17 -fPIC -ffp-contract=off -c $C/seb_sizing.cpp -o $OUT/obj/seb_sizing.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libseb_bloom.so $OUT/obj/*.o -Wl,-rpath,/opt/rocm/lib
echo "$OUT/libseb_bloom.so"
