#!/bin/bash
# Round 4 batch j: resident epochs (experimental module) on the small
# single-rank grids, against the default path.
set -o pipefail
OUT=gpurun_out/${1:-r04j}
mkdir -p "$OUT"
J="$OUT/resident.jsonl"; : > "$J"
run() { timeout -k 10 120 env "$@" >> "$J" 2>> "$OUT/err.log" || { echo "FAILED: $*" >> "$OUT/err.log"; return 1; }; }
B="python bench.py --steps 10 --warmup 2 --verify 60 --no-phase-step"
X="GOL_NATIVE_SO=exp_so/_gol.so"
for rep in 1 2; do
  run GOL_X=0 $B --size 8192 || exit 1
  run $X GOL_RESIDENT=1 $B --size 8192 || exit 1
  run $X GOL_RESIDENT=1 GOL_RES_SYNC=1 $B --size 8192 || exit 1
  run $X GOL_RESIDENT=1 GOL_RES_K=16 $B --size 8192 || exit 1
  run GOL_X=0 $B --size 16384 || exit 1
  run $X GOL_RESIDENT=1 $B --size 16384 || exit 1
  run GOL_X=0 $B --size 4096 || exit 1
  run $X GOL_RESIDENT=1 $B --size 4096 || exit 1
done
