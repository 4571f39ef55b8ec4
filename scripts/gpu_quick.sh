#!/bin/bash
# Smoke, GPU test tier and the driver-argument 1-GPU bench, each under its own limit.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
echo smoke ok
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/b20.json 2>gpurun_out/b20.err
cat gpurun_out/b20.json
