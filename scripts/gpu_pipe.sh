#!/bin/bash
# Pipelined wave pairs (GOL_PIPE): GPU tests, then A/B benches on the full
# grid and the 8-GPU rank tile.  Every GPU step has its own limit.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "pipe" \
  > gpurun_out/pipe_tests.log 2>&1
tail -3 gpurun_out/pipe_tests.log
bash scripts/gpu_ab.sh "base::" "pipe:GOL_PIPE=2:" \
  "tile:GOL_XLANE=-1:--height 4096" "tile-pipe-add12:GOL_PIPE=2 GOL_XLANE=3:--height 4096 --tmax 12" \
  "tile-pipe-add16:GOL_PIPE=2 GOL_XLANE=3:--height 4096 --tmax 16" "tile-pipe-dpp16:GOL_PIPE=2 GOL_XLANE=0:--height 4096 --tmax 16"
