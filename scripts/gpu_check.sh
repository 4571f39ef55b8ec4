#!/bin/bash
# GPU validation pass: smoke, GPU test tier, 1-GPU bench.  Each GPU step has
# its own time limit and the chain stops at the first failure.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/rocm_smi.txt 2>&1 || true
timeout -k 10 600 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > gpurun_out/smoke.log 2>&1
echo "smoke ok"
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
echo "pytest gpu ok"
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
cat gpurun_out/bench.json
