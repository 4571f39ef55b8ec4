#!/bin/bash
# Round 4 batch u: linked launches (with the folded strip) on the 8-GPU rank
# tile, single-rank ring and the multi-rank schedule (one-rank RCCL rehearsal).
set -o pipefail
OUT=gpurun_out/${1:-r04u}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
J="$OUT/ab.jsonl"; : > "$J"
run() { echo "$*" >> "$OUT/progress.log"; timeout -k 10 150 env "$@" >> "$J" 2>> "$OUT/err.log" || { echo "FAILED: $*" >> "$OUT/err.log"; return 1; }; }
B="python bench.py --steps 10 --warmup 2 --verify 60 --no-phase-step --height 4096"
for rep in 1 2 3; do
  run GOL_AB=default $B || exit 1
  run GOL_AB=link GOL_LINK=1 $B || exit 1
  run GOL_AB=default $B --rehearse-rccl || exit 1
  run GOL_AB=link GOL_LINK=1 $B --rehearse-rccl || exit 1
done
