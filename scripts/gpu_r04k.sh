#!/bin/bash
# Round 4 batch k: linked launches (experimental module) across row-ring
# epochs on small single-rank grids, against the default path.
set -o pipefail
OUT=gpurun_out/${1:-r04k}
mkdir -p "$OUT"
J="$OUT/linked.jsonl"; : > "$J"
run() { timeout -k 10 120 env "$@" >> "$J" 2>> "$OUT/err.log" || { echo "FAILED: $*" >> "$OUT/err.log"; return 1; }; }
B="python bench.py --steps 10 --warmup 2 --verify 60 --no-phase-step"
X="GOL_NATIVE_SO=exp_so/_gol.so"
for rep in 1 2; do
  for sz in "--size 4096" "--size 8192" "--size 16384" "--height 4096"; do
    run GOL_X=0 $B $sz || exit 1
    run $X GOL_LINK=1 $B $sz || exit 1
  done
done
