#!/bin/bash
# Short-segment schedule with the adder window (T = 12): correctness, then the
# 8-GPU rank tile (32768 x 4096) A/B against the default.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "short_segment" > gpurun_out/pytest_short.log 2>&1
tail -2 gpurun_out/pytest_short.log
exec_ab() { scripts/gpu_ab.sh "$@"; }
exec_ab "dpp16_h4k::--height 4096" "addshort12_h4k:GOL_XLANE=3 GOL_SHORT=2:--height 4096 --tmax 12" \
  "addshort12_h4k_w4096:GOL_XLANE=3 GOL_SHORT=2 GOL_TARGET_WAVES=4096:--height 4096 --tmax 12" \
  "addshort12_h4k_w3500:GOL_XLANE=3 GOL_SHORT=2 GOL_TARGET_WAVES=3500:--height 4096 --tmax 12"
