#!/bin/bash
# Build libh2s variants for scripts/time_variants.py.
# Usage: bash scripts/build_variants.sh NAME:"-DFLAG ..." NAME2:"..."
# Only the product tile instances (h2s_fast.hip, h2s_fast_lp.hip) are rebuilt
# with the flags;
# every other object comes from the in-tree build (hdr-to-sdr_amd/build/obj,
# run `python -c "import __graft_entry__ as g; g.build()"` first).
# Outputs scripts/variants/libh2s_NAME.so (git-ignored, travels with gpurun).
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/hdr-to-sdr_amd/csrc
O=$ROOT/hdr-to-sdr_amd/build/obj
V=$ROOT/scripts/variants
mkdir -p "$V"
FLAGS="-O3 -std=c++17 -fno-slp-vectorize -fPIC -Wno-unused-value -Wno-unused-result -Wno-pass-failed"
MMC=${MMC-""}   # extra flags for h2s_fast.hip (_build.py SOURCE_FLAGS; env MMC overrides)
pids=()
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  [ "$flags" = "$spec" ] && flags=""
  (
    # DBG=1: the debug instances (h2s_debug_float) get the flags too
    d12="$O/h2s_fast_dbg12.hip.o"; d345="$O/h2s_fast_dbg345.hip.o"
    if [ "${DBG:-0}" = 1 ]; then
      d12="$V/dbg12_$name.o"; d345="$V/dbg345_$name.o"
      /opt/rocm/bin/hipcc --offload-arch=gfx950 $FLAGS $flags -c -o "$d12" "$C/h2s_fast_dbg12.hip" &&
      /opt/rocm/bin/hipcc --offload-arch=gfx950 $FLAGS $flags -c -o "$d345" "$C/h2s_fast_dbg345.hip" || exit 1
    fi
    # KERN=1: h2s_kernels.hip (generic kernel, peak statistics) gets the flags too
    kern="$O/h2s_kernels.hip.o"
    if [ "${KERN:-0}" = 1 ]; then
      kern="$V/kern_$name.o"
      /opt/rocm/bin/hipcc --offload-arch=gfx950 $FLAGS -ffp-contract=off $flags -c -o "$kern" "$C/h2s_kernels.hip" || exit 1
    fi
    /opt/rocm/bin/hipcc --offload-arch=gfx950 $FLAGS $MMC $flags -c -o "$V/fast_$name.o" "$C/h2s_fast.hip" &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 $FLAGS $flags -c -o "$V/fastlp_$name.o" "$C/h2s_fast_lp.hip" &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$V/libh2s_$name.so" "$V/fast_$name.o" "$V/fastlp_$name.o" \
      "$d345" "$d12" "$O/h2s_api.hip.o" "$kern" \
      "$O/h2s_preview.hip.o" "$O/h2s_cube.cpp.o" && rm -f "$V/fast_$name.o" "$V/fastlp_$name.o" "$V/dbg12_$name.o" "$V/dbg345_$name.o" "$V/kern_$name.o"
  ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
ls -la "$V"
