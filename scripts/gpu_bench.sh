#!/bin/bash
# 1-GPU bench with the driver's arguments, per-rank strong-scaling tiles, and
# a kernel-trace profile of the bench.  Each GPU step has its own limit.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 180 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err
cat gpurun_out/bench_driver.json
for h in 16384 8192 4096; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --height $h --epoch 256 > gpurun_out/bench_tile_$h.json 2>> gpurun_out/bench_tiles.err
  cat gpurun_out/bench_tile_$h.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- python3 bench.py --steps 5 --warmup 1 > gpurun_out/prof/bench_trace.json 2> gpurun_out/prof/bench_trace.err
echo trace ok
