set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06_lpab
timeout -k 10 200 env H2S_LIB=$PWD/scripts/variants/libh2s_lattice.so python -u scripts/time_lp_variants_r06.py lattice > gpurun_out/r06_lpab/lattice.log 2>&1 || exit 1
tail -1 gpurun_out/r06_lpab/lattice.log
timeout -k 10 200 env H2S_LP_TAB=0 python -u scripts/time_lp_variants_r06.py table_linear > gpurun_out/r06_lpab/linear.log 2>&1 || exit 1
tail -1 gpurun_out/r06_lpab/linear.log
timeout -k 10 200 env H2S_LP_TAB=1 python -u scripts/time_lp_variants_r06.py table_morton > gpurun_out/r06_lpab/morton.log 2>&1 || exit 1
tail -1 gpurun_out/r06_lpab/morton.log
