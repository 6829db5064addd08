#!/bin/bash
# Build a timing-only variant of libh2s from a patch of the tile kernel
# (profiles/<round>/ab_patches/*.patch), without touching the product source:
# the sources are copied to a scratch directory, the patch applied there, the
# product tile instances (h2s_fast.hip, h2s_fast_lp.hip) rebuilt -- and every
# other translation unit the patch touches, or all of them when it touches a
# header -- and linked with the in-tree objects of everything else (run the
# in-tree build first).
# Usage: bash scripts/build_ablation.sh NAME PATCH|none ["-DFLAG ..."]
# Output: scripts/variants/libh2s_NAME.so (git-ignored, travels with gpurun)
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1
PATCH=/dev/null   # "none": the product source, built with FLAGS only
if [ "$2" != none ]; then PATCH=$(cd "$(dirname "$2")" && pwd)/$(basename "$2"); fi
O=$ROOT/hdr-to-sdr_amd/build/obj
V=$ROOT/scripts/variants
T=$(mktemp -d /tmp/h2s_abl_XXXX)
trap 'rm -rf "$T"' EXIT
mkdir -p "$V" "$T/hdr-to-sdr_amd"
cp -r "$ROOT/hdr-to-sdr_amd/csrc" "$T/hdr-to-sdr_amd/"
cp -r "$ROOT/include" "$T/"
if [ "$PATCH" != /dev/null ]; then (cd "$T" && patch -p1 -s < "$PATCH"); fi
C=$T/hdr-to-sdr_amd/csrc
FLAGS="-O3 -std=c++17 -fno-slp-vectorize -fPIC -Wno-unused-value -Wno-unused-result -Wno-pass-failed -I$T/include ${3:-}"
HDR=0
if grep -q '^+++ .*\.h[[:space:]]' "$PATCH"; then HDR=1; fi
OBJS=()
PIDS=()
for s in h2s_fast_dbg345.hip h2s_fast_dbg12.hip h2s_fast_lp.hip h2s_fast.hip h2s_api.hip h2s_kernels.hip h2s_preview.hip h2s_cube.cpp; do
  if [ $s = h2s_fast.hip ] || [ $s = h2s_fast_lp.hip ] || [ $HDR = 1 ] || grep -q "^+++ .*/$s[[:space:]]" "$PATCH"; then
    extra=""
    if [ $s = h2s_kernels.hip ]; then extra="-ffp-contract=off"; fi
    /opt/rocm/bin/hipcc --offload-arch=gfx950 $FLAGS $extra -c -o "$T/$s.o" "$C/$s" &
    PIDS+=($!)
    OBJS+=("$T/$s.o")
  else
    OBJS+=("$O/$s.o")
  fi
done
for p in "${PIDS[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$V/libh2s_$NAME.so" "${OBJS[@]}"
echo "built $V/libh2s_$NAME.so"
