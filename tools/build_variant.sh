#!/bin/bash
# Build a kernel variant of libdash into tools/variants/libdash_NAME.so (experiments only).
# Usage: tools/build_variant.sh NAME [extra hipcc flags...]
set -euo pipefail
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/ue22cs343bb1-openmp-assignment_amd
OUT=$ROOT/tools/variants; mkdir -p "$OUT"
HIPCC=/opt/rocm/bin/hipcc
$HIPCC --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$ROOT/include" -I"$PKG/csrc" -Wno-bitwise-instead-of-logical \
    "$@" -c -o "$OUT/k_$NAME.o" "${SRC:-$PKG/csrc/dash_kernels.hip}"
$HIPCC --offload-arch=gfx950 -shared -fPIC -o "$OUT/libdash_$NAME.so" "$OUT/k_$NAME.o" "$PKG/build/dash_api.o" "$PKG/build/dash_host.o"
rm -f "$OUT/k_$NAME.o"
echo "built $OUT/libdash_$NAME.so"
