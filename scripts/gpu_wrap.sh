#!/bin/bash
# Wrap mode + folded last strip: the whole GPU tier, then A/B benches on the
# full grid and the 8-GPU rank tile (local fill and RCCL rehearsal).  Every
# GPU step has its own limit.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tier.log 2>&1
tail -n 3 gpurun_out/gpu_tier.log
bash scripts/gpu_ab.sh "wrap::" "nowrap:GOL_WRAP=0:" \
  "t4k-wrap::--height 4096" "t4k-nowrap:GOL_WRAP=0:--height 4096" \
  "r4k-wrap::--height 4096 --rehearse-rccl" "r4k-nowrap:GOL_WRAP=0:--height 4096 --rehearse-rccl" \
  "r16k-wrap::--height 16384 --rehearse-rccl" "r16k-nowrap:GOL_WRAP=0:--height 16384 --rehearse-rccl"
