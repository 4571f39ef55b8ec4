#!/bin/bash
# Kernel trace of the 1-GPU bench on the 8-GPU per-rank tile (32768 x 4096).
set -euo pipefail
export TMPDIR=/tmp
cd /tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/trace -o tile -- \
  python3 $R/bench.py --size 32768 --height 4096 --steps 200 --warmup 20 > $R/gpurun_out/trace/bench.json
find $R/gpurun_out/trace -name '*kernel_stats.csv' | head -1 | xargs cat | head -20
