set -o pipefail
bash tools/gpu_round.sh r02e || exit $?
bash tools/pmc_bench.sh r02e || exit 6
