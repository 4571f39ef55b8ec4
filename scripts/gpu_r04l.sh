#!/bin/bash
# Round 4 batch l: linked launches on by default for small ring tiles: the
# linked-launch and ring tests, then the A/B (GOL_LINK=0 off, -1 default).
set -o pipefail
OUT=gpurun_out/${1:-r04l}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu.py \
  -k "linked or link_launches or row_ring or u8_via_bits" > "$OUT/link_tests.log" 2>&1 || exit $?
J="$OUT/ab.jsonl"; : > "$J"
run() { timeout -k 10 120 env "$@" >> "$J" 2>> "$OUT/err.log" || { echo "FAILED: $*" >> "$OUT/err.log"; return 1; }; }
B="python bench.py --steps 10 --warmup 2 --verify 60 --no-phase-step"
for rep in 1 2 3; do
  for sz in "--size 8192" "--size 8192 --layout u8" "--size 4096" "--height 4096" "--size 16384"; do
    run GOL_LINK=-1 $B $sz || exit 1
    run GOL_LINK=0 $B $sz || exit 1
  done
done
timeout -k 10 120 python bench.py --size 8192 --layout u8 --steps 10 --warmup 2 > "$OUT/bench8192_u8.json" 2>> "$OUT/err.log" || exit 1
