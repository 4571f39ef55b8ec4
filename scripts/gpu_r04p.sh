#!/bin/bash
# Round 4 batch p: one-sided window from one DPP shift + two funnel shifts
# (GOL_ADDER_DPP=1, 3 half-rate VALU ops) vs the carry adder window (4), as a
# level-body microbenchmark and end to end (exp_alt/adddpp/_gol.so).
set -o pipefail
OUT=gpurun_out/${1:-r04p}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 120 ./bin/ubench_vbody > "$OUT/vbody_carry.txt" 2>&1 || exit $?
timeout -k 10 120 ./bin/ubench_vbody_dpp1 > "$OUT/vbody_dpp1.txt" 2>&1 || exit $?
J="$OUT/ab.jsonl"; : > "$J"
run() { echo "$*" >> "$OUT/progress.log"; timeout -k 10 180 env "$@" >> "$J" 2>> "$OUT/err.log" || { echo "FAILED: $*" >> "$OUT/err.log"; return 1; }; }
B="python bench.py --steps 10 --warmup 2 --verify 120 --no-phase-step"
for rep in 1 2 3; do
  for sz in "--size 32768" "--size 16384" "--height 8192"; do
    run GOL_AB=carry $B $sz || exit 1
    run GOL_AB=dpp1 GOL_NATIVE_SO=exp_alt/adddpp/_gol.so $B $sz || exit 1
  done
done
