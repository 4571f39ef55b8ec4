#!/bin/bash
# Round 4 batch x: epoch depth and T of the multi-rank schedule on the 8-GPU
# rank tile now that the blocks of an epoch run linked (one-rank rehearsal).
set -o pipefail
OUT=gpurun_out/${1:-r04x}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
J="$OUT/ab.jsonl"; : > "$J"
run() { echo "$*" >> "$OUT/progress.log"; timeout -k 10 150 env "$@" >> "$J" 2>> "$OUT/err.log" || { echo "FAILED: $*" >> "$OUT/err.log"; return 1; }; }
B="python bench.py --steps 10 --warmup 2 --verify 60 --no-phase-step --height 4096 --rehearse-rccl"
for rep in 1 2; do
  for e in 256 384 512 192; do
    run GOL_AB=e$e $B --epoch $e || exit 1
  done
  run GOL_AB=t12 $B --tmax 12 --epoch 192 || exit 1
  run GOL_AB=t12 $B --tmax 12 --epoch 384 || exit 1
  run GOL_AB=t8 $B --tmax 8 --epoch 256 || exit 1
done
