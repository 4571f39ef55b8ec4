#!/bin/bash
# Round-end style validation on one MI355X: smoke, the whole GPU test tier, the
# default 1-GPU bench, then a rocprofv3 profile of the bench (kernel trace +
# PMC passes) on the 32768^2 grid and on the 8-GPU per-rank tile.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
cat gpurun_out/bench.json
BENCH_ARGS="--steps 500 --warmup 50" bash scripts/profile_bench.sh
mv gpurun_out/prof gpurun_out/prof_full
BENCH_ARGS="--steps 20 --warmup 2 --size 32768 --height 4096" bash scripts/profile_bench.sh
mv gpurun_out/prof gpurun_out/prof_tile
