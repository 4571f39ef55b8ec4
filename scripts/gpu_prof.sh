#!/bin/bash
# rocprofv3 kernel-trace stats of the default bench (full grid and the 8-GPU
# rank tile), then one PMC pass each.  Every GPU step has its own limit.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_full -o run -- python3 bench.py --steps 5 --warmup 1 > gpurun_out/prof_full.json 2> gpurun_out/prof_full.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_tile -o run -- python3 bench.py --steps 5 --warmup 1 --height 4096 > gpurun_out/prof_tile.json 2> gpurun_out/prof_tile.err
bash scripts/pmc_ab.sh "--gpus 1 --steps 3 --warmup 1 --prewarm 1000" "full:"
bash scripts/pmc_ab.sh "--gpus 1 --steps 3 --warmup 1 --prewarm 1000 --height 4096" "tile:"
