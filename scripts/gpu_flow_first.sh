#!/bin/bash
# First GPU pass over the flow kernel: its own tests, then the A/B matrix.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r05
timeout -k 10 400 python -u -m pytest tests/test_gpu_flow.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r05/pytest_flow.log 2>&1 || { tail -50 gpurun_out/r05/pytest_flow.log; exit 1; }
tail -3 gpurun_out/r05/pytest_flow.log
timeout -k 10 900 python -u scripts/bench_matrix.py scripts/matrices/r05_flow_first.txt gpurun_out/r05/flow_first.jsonl --timeout 120
