#!/bin/bash
# Build a kernel variant of libdash into tools/variants/libdash_NAME.so (experiments only).
# Usage: [SRC=file.hip] [PATCHES="tools/experiments/x.patch ..."] tools/build_variant.sh NAME [extra hipcc flags...]
# PATCHES are applied to a temporary copy of the kernel source (e.g. issue_probes.patch: the
# DASH_PAD_VALU / DASH_PAD_SALU / DASH_PAD_VHALF issue-cost probes and DASH_HEADLINE_ONLY).
set -euo pipefail
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/ue22cs343bb1-openmp-assignment_amd
OUT=${OUT:-$ROOT/tools/variants}; mkdir -p "$OUT"
HIPCC=/opt/rocm/bin/hipcc
SRC=${SRC:-$PKG/csrc/dash_kernels.hip}
if [ -n "${PATCHES:-}" ]; then
    TMP=$(mktemp -d); cp "$SRC" "$TMP/dash_kernels.hip"
    for p in $PATCHES; do patch -s "$TMP/dash_kernels.hip" "$ROOT/$p"; done
    SRC=$TMP/dash_kernels.hip
fi
$HIPCC --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$ROOT/include" -I"$PKG/csrc" -Wno-bitwise-instead-of-logical -Wno-pass-failed \
    -DDASH_WAVES_PER_EU=5 "$@" -c -o "$OUT/k_$NAME.o" "$SRC"
$HIPCC --offload-arch=gfx950 -shared -fPIC -o "$OUT/libdash_$NAME.so" "$OUT/k_$NAME.o" "$PKG/build/dash_api.o" "$PKG/build/dash_host.o"
rm -f "$OUT/k_$NAME.o"
echo "built $OUT/libdash_$NAME.so"
