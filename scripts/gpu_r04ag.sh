#!/bin/bash
# Round 4 batch ag: termination-poll interval on linked small tiles (every
# poll joins the two streams): 8192^2 and the 8-GPU rank tile.
set -o pipefail
OUT=gpurun_out/${1:-r04ag}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
J="$OUT/ab.jsonl"; : > "$J"
run() { echo "$*" >> "$OUT/progress.log"; timeout -k 10 150 env "$@" >> "$J" 2>> "$OUT/err.log" || { echo "FAILED: $*" >> "$OUT/err.log"; return 1; }; }
B="python bench.py --steps 10 --warmup 2 --verify 60 --no-phase-step"
for rep in 1 2 3; do
  for p in 256 512 1024; do
    run GOL_AB=p$p $B --size 8192 --poll $p || exit 1
  done
  for p in 512 1024; do
    run GOL_AB=p$p $B --height 4096 --rehearse-rccl --poll $p || exit 1
  done
done
