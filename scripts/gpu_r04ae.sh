#!/bin/bash
# Round 4 batch ae: 4-wave vs 8-wave groups (GOL_GROUP=4 vs default 8) for
# the adder T = 12 tiles: 32768^2, the 2- and 4-GPU rank tiles (rehearsal),
# 16384^2 (65536^2 left out: see bench.py ORACLE_WHOLE_CELLS).
set -o pipefail
OUT=gpurun_out/${1:-r04ae}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
J="$OUT/ab.jsonl"; : > "$J"
run() { echo "$*" >> "$OUT/progress.log"; timeout -k 10 200 env "$@" >> "$J" 2>> "$OUT/err.log" || { echo "FAILED: $*" >> "$OUT/err.log"; return 1; }; }
B="python bench.py --steps 10 --warmup 2 --verify 60 --no-phase-step"
for rep in 1 2 3; do
  for sz in "--size 32768" "--height 16384 --rehearse-rccl" "--height 8192 --rehearse-rccl" "--size 16384"; do
    run GOL_AB=g8 $B $sz || exit 1
    run GOL_AB=g4 GOL_GROUP=4 $B $sz || exit 1
  done
done
