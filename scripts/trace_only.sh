#!/bin/bash
# Kernel trace of one bench configuration: BENCH_ARGS, output dir $1.
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/trace}
mkdir -p $OUT
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 bench.py $BENCH_ARGS > $OUT/bench.json 2> $OUT/bench.err
echo "trace $OUT ok"
