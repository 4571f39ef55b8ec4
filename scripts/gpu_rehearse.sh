#!/bin/bash
# One-GPU rehearsal of the N-GPU strong-scaling ranks: the per-rank tile
# (32768 x 32768/N) with the multi-rank schedule (epoch 16T, early-boundary
# overlap) exchanging with itself over a 1-rank RCCL communicator.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "rehearsal or rccl or multi_subdomain or adder_window_row" > gpurun_out/pytest_rehearse.log 2>&1
tail -1 gpurun_out/pytest_rehearse.log
scripts/gpu_ab.sh \
  "tile8_plain::--height 4096 --epoch 256" \
  "tile8_rccl_off::--height 4096 --rehearse-rccl --overlap off" \
  "tile8_rccl_on::--height 4096 --rehearse-rccl --overlap on" \
  "tile8_rccl_auto::--height 4096 --rehearse-rccl" \
  "tile4_rccl_off::--height 8192 --rehearse-rccl --overlap off" \
  "tile4_rccl_auto::--height 8192 --rehearse-rccl" \
  "tile2_rccl_off::--height 16384 --rehearse-rccl --overlap off" \
  "tile2_rccl_auto::--height 16384 --rehearse-rccl"
