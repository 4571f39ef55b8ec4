#!/bin/bash
# Round 4 batch d: GPU tier (row ring, 4-wave groups at small T), then the
# row ring's A/B on the single-rank grids.
set -o pipefail
OUT=gpurun_out/${1:-r04d}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu.py \
  -k "row_ring" > "$OUT/ring_tests.log" 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests \
  --deselect tests/test_rccl_multirank.py > "$OUT/tier.log" 2>&1 || exit $?
J="$OUT/ab.jsonl"; : > "$J"
run() { timeout -k 10 120 env "$@" >> "$J" 2>> "$OUT/err.log" || { echo "FAILED: $*" >> "$OUT/err.log"; return 1; }; }
B="python bench.py --steps 10 --warmup 2 --verify 0 --no-phase-step"
for rep in 1 2 3; do
  for ring in 1 0; do
    run GOL_ROW_RING=$ring $B --size 8192 || exit 1
    run GOL_ROW_RING=$ring $B --size 8192 --layout u8 || exit 1
    run GOL_ROW_RING=$ring $B --size 32768 || exit 1
  done
done
for rep in 1 2; do
  run GOL_ROW_RING=1 $B --size 16384 || exit 1
  run GOL_ROW_RING=0 $B --size 16384 || exit 1
  run GOL_ROW_RING=1 $B --size 65536 --steps 3 || exit 1
  run GOL_ROW_RING=0 $B --size 65536 --steps 3 || exit 1
done
timeout -k 10 120 python bench.py --size 8192 --layout u8 --steps 10 --warmup 2 > "$OUT/bench8192_u8.json" 2>> "$OUT/err.log" || exit 1
timeout -k 10 200 python bench.py > "$OUT/bench_default.json" 2>> "$OUT/err.log" || exit 1
