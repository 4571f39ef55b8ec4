#!/bin/bash
# Round 4: small-grid (8192^2, BASELINE config 2) temporal-block depth and
# window sweep, bit and byte layouts.  One JSON line per configuration.
set -o pipefail
OUT=gpurun_out/${1:-r04_small}
mkdir -p "$OUT"
J="$OUT/small.jsonl"
: > "$J"
run() {  # env..., then bench args
  timeout -k 10 120 env "$@" >> "$J" 2>> "$OUT/err.log" || { echo "FAILED: $*" >> "$OUT/err.log"; return 1; }
}
B="python bench.py --size 8192 --steps 10 --warmup 2 --verify 0 --no-phase-step"
for rep in 1 2; do
  for x in -1 0 3; do
    for t in 2 4 8 12 16; do
      [ "$x" = "3" ] && [ "$t" = "16" ] && continue
      run GOL_XLANE=$x $B --layout bits --tmax $t || exit 1
    done
  done
  run GOL_XLANE=-1 $B --layout bits || exit 1
  run GOL_XLANE=-1 $B --layout u8 || exit 1
  run GOL_U8_KERNEL=lds $B --layout u8 --u8-compute bytes || exit 1
done
