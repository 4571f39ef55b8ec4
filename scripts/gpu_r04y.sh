#!/bin/bash
# Round 4 batch y: shallower linked blocks on the 8-GPU rank tile in the
# multi-rank schedule (forced GOL_LINK=1 with an explicit T).
set -o pipefail
OUT=gpurun_out/${1:-r04y}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
J="$OUT/ab.jsonl"; : > "$J"
run() { echo "$*" >> "$OUT/progress.log"; timeout -k 10 150 env "$@" >> "$J" 2>> "$OUT/err.log" || { echo "FAILED: $*" >> "$OUT/err.log"; return 1; }; }
B="python bench.py --steps 10 --warmup 2 --verify 60 --no-phase-step --height 4096 --rehearse-rccl"
for rep in 1 2; do
  run GOL_AB=default $B || exit 1
  run GOL_AB=l12 GOL_LINK=1 $B --tmax 12 --epoch 192 || exit 1
  run GOL_AB=l12 GOL_LINK=1 $B --tmax 12 --epoch 384 || exit 1
  run GOL_AB=l8 GOL_LINK=1 $B --tmax 8 --epoch 128 || exit 1
  run GOL_AB=l8 GOL_LINK=1 $B --tmax 8 --epoch 256 || exit 1
done
