#!/bin/bash
# Side-stream termination polls (own RCCL communicator): RCCL GPU tests, then
# A/B in the one-GPU RCCL rehearsal of the 2/4/8-GPU rank tiles.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "rccl or rehears" > gpurun_out/sidepoll_tests.log 2>&1
tail -n 2 gpurun_out/sidepoll_tests.log
bash scripts/gpu_ab.sh "r4k-side::--height 4096 --rehearse-rccl" "r4k-comp:GOL_SIDE_POLL=0:--height 4096 --rehearse-rccl" \
  "r8k-side::--height 8192 --rehearse-rccl" "r8k-comp:GOL_SIDE_POLL=0:--height 8192 --rehearse-rccl" \
  "r16k-side::--height 16384 --rehearse-rccl" "r16k-comp:GOL_SIDE_POLL=0:--height 16384 --rehearse-rccl"
