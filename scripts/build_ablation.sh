#!/bin/bash
# Build a timing-only variant of libh2s from a patch of the tile kernel
# (profiles/<round>/ab_patches/*.patch), without touching the product source:
# the sources are copied to a scratch directory, the patch applied there, the
# product tile instances (h2s_fast.hip, h2s_fast_lp.hip) rebuilt -- and
# h2s_kernels.hip when the patch touches it -- and linked with the in-tree
# objects of everything else (run the in-tree build first).
# Usage: bash scripts/build_ablation.sh NAME PATCH ["-DFLAG ..."]
# Output: scripts/variants/libh2s_NAME.so (git-ignored, travels with gpurun)
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1
PATCH=$(cd "$(dirname "$2")" && pwd)/$(basename "$2")
O=$ROOT/hdr-to-sdr_amd/build/obj
V=$ROOT/scripts/variants
T=$(mktemp -d /tmp/h2s_abl_XXXX)
trap 'rm -rf "$T"' EXIT
mkdir -p "$V" "$T/hdr-to-sdr_amd"
cp -r "$ROOT/hdr-to-sdr_amd/csrc" "$T/hdr-to-sdr_amd/"
cp -r "$ROOT/include" "$T/"
(cd "$T" && patch -p1 -s < "$PATCH")
C=$T/hdr-to-sdr_amd/csrc
FLAGS="-O3 -std=c++17 -fno-slp-vectorize -fPIC -Wno-unused-value -Wno-unused-result -Wno-pass-failed -I$T/include ${3:-}"
/opt/rocm/bin/hipcc --offload-arch=gfx950 $FLAGS -c -o "$T/fast.o" "$C/h2s_fast.hip" &
/opt/rocm/bin/hipcc --offload-arch=gfx950 $FLAGS -c -o "$T/fastlp.o" "$C/h2s_fast_lp.hip" &
KO=$O/h2s_kernels.hip.o
if grep -q '^+++ .*h2s_kernels.hip' "$PATCH"; then
  KO=$T/kernels.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 $FLAGS -ffp-contract=off -c -o "$KO" "$C/h2s_kernels.hip" &
fi
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$V/libh2s_$NAME.so" "$T/fast.o" "$T/fastlp.o" \
  "$O/h2s_fast_dbg345.hip.o" "$O/h2s_fast_dbg12.hip.o" "$O/h2s_api.hip.o" "$KO" \
  "$O/h2s_preview.hip.o" "$O/h2s_cube.cpp.o"
echo "built $V/libh2s_$NAME.so"
