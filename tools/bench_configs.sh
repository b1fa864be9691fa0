#!/bin/bash
# Bench lines + rocprofv3 kernel stats for BASELINE configs[1] and configs[4] (per-GPU share).
# Usage: tools/bench_configs.sh TAG
set -o pipefail
TAG=${1:-x}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
C1="--batch 1024 --dtype fp32 --loss infonce"
C4="--hidden 512 --seq 128"
timeout -k 10 400 python bench.py $C1 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_c1_$TAG.json 2> $OUT/bench_c1_$TAG.err || { echo c1 failed; exit 1; }
timeout -k 10 600 python bench.py $C4 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_c4_$TAG.json 2> $OUT/bench_c4_$TAG.err || { echo c4 failed; exit 2; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c1_$TAG -o prof -- python $ROOT/bench.py $C1 --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2>&1 || { echo c1 prof failed; exit 3; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4_$TAG -o prof -- python $ROOT/bench.py $C4 --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || { echo c4 prof failed; exit 4; }
echo configs done
