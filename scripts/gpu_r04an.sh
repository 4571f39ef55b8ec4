#!/bin/bash
# Round 4 batch an: final round-4 numbers across grid sizes and the rank tiles
# of the strong-scaling split (one-rank RCCL rehearsal), all verified.
set -o pipefail
OUT=gpurun_out/${1:-r04an}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
J="$OUT/final_sizes.jsonl"; : > "$J"
run() { echo "$*" >> "$OUT/progress.log"; timeout -k 10 300 env "$@" >> "$J" 2>> "$OUT/err.log" || { echo "FAILED: $*" >> "$OUT/err.log"; return 1; }; }
B="python bench.py --steps 10 --warmup 2 --verify 60 --no-phase-step"
for rep in 1 2; do
  for sz in "--size 4096" "--size 8192" "--size 8192 --layout u8" "--size 16384" "--size 32768" "--size 32768 --layout u8" \
            "--height 16384 --rehearse-rccl" "--height 8192 --rehearse-rccl" "--height 4096 --rehearse-rccl"; do
    run GOL_AB=final $B $sz || exit 1
  done
done
run GOL_AB=final python bench.py --steps 3 --warmup 1 --verify 30 --no-phase-step --size 65536 || exit 1
