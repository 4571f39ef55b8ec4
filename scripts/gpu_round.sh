#!/bin/bash
# One GPU validation + measurement pass: smoke, GPU test tier, bench sweep.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
SWEEP_TIMEOUT=200 timeout -k 10 900 python scripts/sweep.py ${SWEEP_SPEC:-scripts/sweep15.txt} gpurun_out/sweep.jsonl
