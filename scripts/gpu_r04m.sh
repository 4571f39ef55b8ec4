#!/bin/bash
# Round 4 batch m: temporal depth x linked launches on the small grids
# (8192^2, 4096^2, 16384^2): does linking make deeper blocks pay?
set -o pipefail
OUT=gpurun_out/${1:-r04m}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
J="$OUT/sweep.jsonl"; : > "$J"
run() { echo "$*" >> "$OUT/progress.log"; timeout -k 10 120 env "$@" >> "$J" 2>> "$OUT/err.log" || { echo "FAILED: $*" >> "$OUT/err.log"; return 1; }; }
B="python bench.py --steps 10 --warmup 2 --verify 60 --no-phase-step"
for rep in 1 2; do
  run GOL_LINK=-1 $B --size 8192 || exit 1
  for t in 16 12 8; do
    run GOL_LINK=1 $B --size 8192 --tmax $t || exit 1
    run GOL_LINK=1 GOL_GROUP_SMALL=8 $B --size 8192 --tmax $t || exit 1
  done
  run GOL_LINK=1 $B --size 4096 || exit 1
  run GOL_LINK=1 $B --size 4096 --tmax 4 || exit 1
  run GOL_LINK=-1 $B --size 4096 || exit 1
  run GOL_LINK=1 $B --size 16384 || exit 1
  run GOL_LINK=1 $B --size 16384 --tmax 16 || exit 1
  run GOL_LINK=-1 $B --size 16384 || exit 1
done
