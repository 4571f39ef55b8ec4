#!/bin/bash
# Round 4 batch aa: planner wave target of linked launches on the 8-GPU rank
# tile (multi-rank schedule, one-rank rehearsal) and on 8192^2.
set -o pipefail
OUT=gpurun_out/${1:-r04aa}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
J="$OUT/ab.jsonl"; : > "$J"
run() { echo "$*" >> "$OUT/progress.log"; timeout -k 10 150 env "$@" >> "$J" 2>> "$OUT/err.log" || { echo "FAILED: $*" >> "$OUT/err.log"; return 1; }; }
B="python bench.py --steps 10 --warmup 2 --verify 60 --no-phase-step"
for rep in 1 2; do
  for tw in 0 1536 2048 3072 4096; do
    run GOL_AB=tw$tw GOL_TARGET_WAVES=$tw $B --height 4096 --rehearse-rccl || exit 1
    run GOL_AB=tw$tw GOL_TARGET_WAVES=$tw $B --size 8192 || exit 1
  done
done
