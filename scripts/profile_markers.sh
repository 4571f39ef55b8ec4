#!/bin/bash
# roctx marker + kernel trace of the 1-GPU bench (no counters in this pass):
# engine phases (gol.run / gol.halo_exchange / gol.poll_wait) next to the
# per-kernel time.  Full grid and the 8-GPU per-rank tile.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/mk
for cfg in "full:--size 32768" "tile:--size 32768 --height 4096"; do
  name=${cfg%%:*}
  args=${cfg#*:}
  timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv \
    -d gpurun_out/mk/$name -o run -- python3 bench.py --steps 20 --warmup 2 $args \
    > gpurun_out/mk/$name.json 2> gpurun_out/mk/$name.err
  echo "$name ok"
done
find gpurun_out/mk -name "*stats.csv"
