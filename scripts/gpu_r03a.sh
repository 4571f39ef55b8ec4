#!/bin/bash
# Round 3, first GPU pass: the new multi-rank RCCL tests (ranks sharing one
# GPU), device-affinity checks, the full GPU tier, and the default bench with
# its verification gate and per-phase step.  Every GPU step has its own limit.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03a
timeout -k 10 400 python -u -m pytest tests/test_rccl_multirank.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r03a/pytest_multirank.log 2>&1
echo multirank ok
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  --deselect tests/test_rccl_multirank.py > gpurun_out/r03a/pytest_gpu.log 2>&1
tail -2 gpurun_out/r03a/pytest_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/r03a/bench.json 2> gpurun_out/r03a/bench.err
cat gpurun_out/r03a/bench.json
