#!/bin/bash
# Kernel trace of the 1-GPU bench on the per-rank tiles; idle gaps between launches.
set -euo pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for h in ${GAP_HEIGHTS:-4096}; do
  mkdir -p $R/gpurun_out/gaps/h$h
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/gaps/h$h -o run -- \
    python3 $R/bench.py --size 32768 --height $h --steps 5 --warmup 1 > $R/gpurun_out/gaps/h$h/bench.json
  f=$(find $R/gpurun_out/gaps/h$h -name '*kernel_trace.csv' | head -1)
  python3 $R/scripts/launch_gaps.py $f | tee $R/gpurun_out/gaps/h$h/gaps.txt
done
