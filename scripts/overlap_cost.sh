#!/bin/bash
# Cost of the overlapped epoch on the 8-GPU per-rank tile shape, measured with
# 2 in-process ranks on one GPU (32768 x 8192 grid -> two 32768 x 4096 tiles).
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ovl
for ov in off on; do
  for ep in 64 32 16; do
    timeout -k 10 300 ./bin/gol 32768 8192 none --random 1 --engine hip --ranks 2 --comm thread --decomp 1x2 \
      --gens 1000 --no-similarity --overlap $ov --epoch $ep --output none --metrics-json gpurun_out/ovl/m_${ov}_${ep}.json > /dev/null
    python3 -c "import json;m=json.load(open('gpurun_out/ovl/m_${ov}_${ep}.json'));print('overlap=$ov epoch=$ep', 'loop_ms=%.2f'%m['loop_ms'], 'cups=%.3e'%m['cell_updates_per_s'])"
  done
done
