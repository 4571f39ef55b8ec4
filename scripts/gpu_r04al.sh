#!/bin/bash
# Round 4 batch al: linked launches without the per-launch cross-stream event
# (default now) vs with it (GOL_LINK_EVENTS=1): linked and ring tests, the
# rank-tile multi-rank test, then the A/B.
set -o pipefail
OUT=gpurun_out/${1:-r04al}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu.py \
  -k "linked or link_launches or row_ring or links_by_default or u8_via_bits" > "$OUT/link_tests.log" 2>&1 || exit $?
J="$OUT/ab.jsonl"; : > "$J"
run() { echo "$*" >> "$OUT/progress.log"; timeout -k 10 150 env "$@" >> "$J" 2>> "$OUT/err.log" || { echo "FAILED: $*" >> "$OUT/err.log"; return 1; }; }
B="python bench.py --steps 10 --warmup 2 --verify 60 --no-phase-step"
for rep in 1 2 3; do
  for sz in "--size 8192" "--size 8192 --layout u8" "--height 4096" "--height 4096 --rehearse-rccl"; do
    run GOL_AB=noev $B $sz || exit 1
    run GOL_AB=ev GOL_LINK_EVENTS=1 $B $sz || exit 1
  done
done
