#!/bin/bash
# Round 4 batch ad: the adder T = 12 grouped kernel held to 96 VGPRs (5 waves
# per SIMD, 76 B/lane of spills; exp_alt/w5) vs the default 120 (4 waves), on
# 32768^2 with 8-wave groups (default) and 4-wave groups (GOL_GROUP=4).
set -o pipefail
OUT=gpurun_out/${1:-r04ad}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
J="$OUT/ab.jsonl"; : > "$J"
run() { echo "$*" >> "$OUT/progress.log"; timeout -k 10 150 env "$@" >> "$J" 2>> "$OUT/err.log" || { echo "FAILED: $*" >> "$OUT/err.log"; return 1; }; }
B="python bench.py --steps 10 --warmup 2 --verify 60 --no-phase-step"
for rep in 1 2; do
  run GOL_AB=base $B || exit 1
  run GOL_AB=base_g4 GOL_GROUP=4 $B || exit 1
  run GOL_AB=w5 GOL_NATIVE_SO=exp_alt/w5/_gol.so $B || exit 1
  run GOL_AB=w5_g4 GOL_GROUP=4 GOL_NATIVE_SO=exp_alt/w5/_gol.so $B || exit 1
done
