#!/bin/bash
# Round 4 batch aj: host time per block (GOL_HOST_PROFILE=1) on the small grids.
set -o pipefail
OUT=gpurun_out/${1:-r04aj}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
B="python bench.py --steps 10 --warmup 2 --verify 0 --no-phase-step"
for args in "--size 8192" "--size 8192 --height 2048 --tmax 8" "--size 8192 --tmax 8" "--height 4096"; do
  echo "== $args" >> "$OUT/prof.txt"
  timeout -k 10 150 env GOL_HOST_PROFILE=1 $B $args >> "$OUT/prof.txt" 2> "$OUT/err.txt" || exit 1
  grep "host profile" "$OUT/err.txt" >> "$OUT/prof.txt"
done
