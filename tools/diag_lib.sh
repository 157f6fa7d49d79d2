#!/bin/bash
# Build a diagnostic variant of libseb_bloom.so into tools/ab_lib/NAME/ (CPU, here): the product
# sources are copied, the given tools/diag/*.patch files applied to the copy, extra -D flags passed
# to hipcc.  The product sources carry no diagnostic code paths.
#   tools/diag_lib.sh NAME [PATCH...] [-- -DFLAG...]      e.g. tools/diag_lib.sh nogather phase_no_gather
# Run it on the box with SEB_LIB_PATH=tools/ab_lib/NAME/libseb_bloom.so.
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/tools/ab_lib/$NAME
SRC=$OUT/src
rm -rf "$SRC" && mkdir -p "$OUT/obj" "$SRC/storage-engines_amd/csrc" "$SRC/include"
cp "$ROOT"/storage-engines_amd/csrc/*.{hip,h,cpp} "$SRC/storage-engines_amd/csrc/"
cp "$ROOT"/include/*.h "$SRC/include/"
FLAGS=()
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then shift; FLAGS=("$@"); break; fi
  patch -s -d "$SRC" -p1 < "$ROOT/tools/diag/$1.patch"
  shift
done
C=$SRC/storage-engines_amd/csrc
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function ${FLAGS[*]}"
for f in seb_kernels seb_bucket seb_varlen seb_multiget seb_codec; do
  /opt/rocm/bin/hipcc $FL -c $C/$f.hip -o $OUT/obj/$f.o &
done
/opt/rocm/bin/hipcc $FL -c $C/seb_host.cpp -o $OUT/obj/seb_host.o &
g++ -O2 -std=c++17 -fPIC -ffp-contract=off -c $C/seb_sizing.cpp -o $OUT/obj/seb_sizing.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libseb_bloom.so $OUT/obj/*.o -Wl,-rpath,/opt/rocm/lib
echo "$OUT/libseb_bloom.so"
