#!/bin/bash
# Round 4 batch am: the experimental module (rebuilt on the final tree).
set -o pipefail
OUT=gpurun_out/${1:-r04am}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
GOL_NATIVE_SO=exp_so/_gol.so timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  -m "gpu and experimental" tests/test_gpu.py > "$OUT/experimental.log" 2>&1
