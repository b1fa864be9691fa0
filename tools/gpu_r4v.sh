# final build: GPU suite, smoke, bench lines, kernel stats (r4n), then the PMC passes
bash tools/gpu_r4n.sh || exit 1
cd $GRAFT_REPO_ROOT && TT_GRU_XC_COOP=0 bash tools/pmc_bench.sh v
