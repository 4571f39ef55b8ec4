#!/bin/bash
# Round 4 batch t: linked T = 8 launches in 4-wave groups (default) vs 8-wave
# groups (GOL_GROUP_SMALL=8), with the folded strip; T = 12 linked; 4096^2.
set -o pipefail
OUT=gpurun_out/${1:-r04t}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu.py \
  -k "linked or link_launches or row_ring" > "$OUT/link_tests.log" 2>&1 || exit $?
J="$OUT/ab.jsonl"; : > "$J"
run() { echo "$*" >> "$OUT/progress.log"; timeout -k 10 120 env "$@" >> "$J" 2>> "$OUT/err.log" || { echo "FAILED: $*" >> "$OUT/err.log"; return 1; }; }
B="python bench.py --steps 10 --warmup 2 --verify 60 --no-phase-step"
for rep in 1 2 3; do
  run GOL_AB=m4 $B --size 8192 || exit 1
  run GOL_AB=m8 GOL_GROUP_SMALL=8 $B --size 8192 || exit 1
  run GOL_AB=m4 $B --size 8192 --layout u8 || exit 1
  run GOL_AB=m8 GOL_GROUP_SMALL=8 $B --size 8192 --layout u8 || exit 1
  run GOL_AB=t12 GOL_LINK=1 $B --size 8192 --tmax 12 || exit 1
  run GOL_AB=default $B --size 4096 || exit 1
  run GOL_AB=link GOL_LINK=1 $B --size 4096 || exit 1
done
