# A/B: a block's 8 tiles as a 4 x 2 patch (H2S_PATCH_WALK) against the 1 x 8
# row walk -- C2 (timing, output identity) and C3 (timing, parity counts)
set -u -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r05_patch
V=scripts/variants
KINDS=smooth,uniform,website timeout -k 10 500 python -u scripts/time_variants.py $V/libh2s_base.so $V/libh2s_patch.so $V/libh2s_base.so $V/libh2s_patch.so > gpurun_out/r05_patch/c2.log 2>&1 || { tail -8 gpurun_out/r05_patch/c2.log; exit 1; }
cat gpurun_out/r05_patch/c2.log
timeout -k 10 400 python -u scripts/time_lp_variants.py $V/libh2s_base.so $V/libh2s_patch.so $V/libh2s_base.so $V/libh2s_patch.so > gpurun_out/r05_patch/c3.log 2>&1 || { tail -5 gpurun_out/r05_patch/c3.log; exit 1; }
cat gpurun_out/r05_patch/c3.log
