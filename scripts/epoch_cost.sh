#!/bin/bash
# Epoch depth D trade-off on the 8-GPU per-rank tile shape: 1 rank (local
# periodic fill) and 2 in-process ranks on one GPU (device-to-device halo
# copies through the thread transport).
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ep
for ep in 32 64 128 192 256; do
  timeout -k 10 300 python bench.py --size 32768 --height 4096 --epoch $ep > gpurun_out/ep/b_$ep.json
  python3 -c "import json;m=json.load(open('gpurun_out/ep/b_$ep.json'));print('1 rank  epoch=$ep', 'us/gen=%.2f'%(m['ms_per_step']*1e3))"
  timeout -k 10 300 ./bin/gol 32768 8192 none --random 1 --engine hip --ranks 2 --comm thread --decomp 1x2 \
      --gens 1000 --no-similarity --epoch $ep --output none --metrics-json gpurun_out/ep/m_$ep.json > /dev/null
  python3 -c "import json;m=json.load(open('gpurun_out/ep/m_$ep.json'));print('2 ranks epoch=$ep', 'loop_ms=%.2f'%m['loop_ms'])"
done
