#!/bin/bash
# Iteration loop on the GPU box: GPU test tier, then a bench sweep.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
python scripts/sweep.py ${SWEEP_SPEC:-scripts/sweep1.txt} gpurun_out/sweep.jsonl
