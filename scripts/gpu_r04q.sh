#!/bin/bash
# Round 4 batch q: the one-sided window (drifting frame) on the low-occupancy
# tiles, carry form vs one DPP shift (exp_alt/adddpp), forced GOL_XLANE=3.
set -o pipefail
OUT=gpurun_out/${1:-r04q}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
J="$OUT/ab.jsonl"; : > "$J"
run() { echo "$*" >> "$OUT/progress.log"; timeout -k 10 180 env "$@" >> "$J" 2>> "$OUT/err.log" || { echo "FAILED: $*" >> "$OUT/err.log"; return 1; }; }
B="python bench.py --steps 10 --warmup 2 --verify 120 --no-phase-step"
for rep in 1 2; do
  for sz in "--height 4096" "--size 8192"; do
    run GOL_AB=default $B $sz || exit 1
    for t in 16 12 8; do
      run GOL_AB=carry GOL_XLANE=3 $B $sz --tmax $t || exit 1
      run GOL_AB=dpp1 GOL_XLANE=3 GOL_NATIVE_SO=exp_alt/adddpp/_gol.so $B $sz --tmax $t || exit 1
    done
  done
done
