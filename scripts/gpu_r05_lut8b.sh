# LP lut3d-table A/B, second take (the first build had the macro default
# defined after its use: both variants ran the per-pixel form): PMC counts,
# then timing + parity counts
set -u -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
V=scripts/variants
bash scripts/gpu_pmc_ab.sh pmc_lut8b $V/libh2s_base.so $V/libh2s_tab.so || exit 1
cd "$R"
mkdir -p gpurun_out/r05_lut8b
timeout -k 10 400 python -u scripts/time_lp_variants.py $V/libh2s_base.so $V/libh2s_tab.so $V/libh2s_base.so $V/libh2s_tab.so > gpurun_out/r05_lut8b/lp.log 2>&1 || { tail -5 gpurun_out/r05_lut8b/lp.log; exit 1; }
cat gpurun_out/r05_lut8b/lp.log
