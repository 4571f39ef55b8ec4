#!/bin/bash
# Round 4 batch ao: where the linked kernel's write-through tax comes from, on
# tiles whose launches fill the GPU (never linked: GOL_LINK=1 GOL_LINK_FORCE=1
# runs the linked kernel unlinked): sc1 loads and stores, loads plain
# (exp_alt/noload) or stores plain (exp_alt/nostore), against the default.
set -o pipefail
OUT=gpurun_out/${1:-r04ao}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
J="$OUT/ab.jsonl"; : > "$J"
run() { echo "$*" >> "$OUT/progress.log"; timeout -k 10 200 env "$@" >> "$J" 2>> "$OUT/err.log" || { echo "FAILED: $*" >> "$OUT/err.log"; return 1; }; }
B="python bench.py --steps 10 --warmup 2 --verify 60 --no-phase-step"
for rep in 1 2; do
  for sz in "--size 16384" "--size 32768"; do
    run GOL_AB=default $B $sz || exit 1
    run GOL_AB=sc1 GOL_LINK=1 GOL_LINK_FORCE=1 $B $sz || exit 1
    run GOL_AB=noload GOL_LINK=1 GOL_LINK_FORCE=1 GOL_NATIVE_SO=exp_alt/noload/_gol.so $B $sz || exit 1
    run GOL_AB=nostore GOL_LINK=1 GOL_LINK_FORCE=1 GOL_NATIVE_SO=exp_alt/nostore/_gol.so $B $sz || exit 1
  done
done
