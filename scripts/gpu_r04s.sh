#!/bin/bash
# Round 4 batch s: linked launches keep the folded last strip.  Linked and
# ring tests, then 8192^2 bits/u8 (linked by default) three times each.
set -o pipefail
OUT=gpurun_out/${1:-r04s}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu.py \
  -k "linked or link_launches or row_ring" > "$OUT/link_tests.log" 2>&1 || exit $?
J="$OUT/ab.jsonl"; : > "$J"
run() { echo "$*" >> "$OUT/progress.log"; timeout -k 10 120 env "$@" >> "$J" 2>> "$OUT/err.log" || { echo "FAILED: $*" >> "$OUT/err.log"; return 1; }; }
B="python bench.py --steps 10 --warmup 2 --verify 60 --no-phase-step"
for rep in 1 2 3; do
  run GOL_AB=fold $B --size 8192 || exit 1
  run GOL_AB=fold $B --size 8192 --layout u8 || exit 1
done
