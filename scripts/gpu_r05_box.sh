# A/B: the LDS-staged lattice box (H2S_LDS_BOX) on C2 -- timing and output
# identity against the default build, smooth / uniform / website content
set -u -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r05_box
V=scripts/variants
KINDS=smooth,uniform,website timeout -k 10 500 python -u scripts/time_variants.py $V/libh2s_base.so $V/libh2s_box.so $V/libh2s_base.so $V/libh2s_box.so > gpurun_out/r05_box/ab.log 2>&1 || { tail -8 gpurun_out/r05_box/ab.log; exit 1; }
cat gpurun_out/r05_box/ab.log
