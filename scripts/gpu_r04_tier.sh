#!/bin/bash
# Round-4 GPU tier: new tests first (graph keying under drift, 8-rank RCCL,
# the N = 8 bench rehearsal), then the whole GPU tier.
set -o pipefail
OUT=gpurun_out/${1:-r04a}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu.py -k "graphs_survive_drift or graphs_and_chunked" > "$OUT/new_graph.log" 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -v --timeout 700 --timeout-method thread -m gpu \
  tests/test_rccl_multirank.py > "$OUT/multirank.log" 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests \
  --deselect tests/test_rccl_multirank.py > "$OUT/tier.log" 2>&1 || exit $?
