#!/bin/bash
# Round 4 batch v: linked launches wherever two launches fit (rank tiles and
# the multi-rank schedule too).  Whole GPU tier, then default vs GOL_LINK=0.
set -o pipefail
OUT=gpurun_out/${1:-r04v}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 700 --timeout-method thread -m gpu tests \
  > "$OUT/tier.log" 2>&1 || exit $?
J="$OUT/ab.jsonl"; : > "$J"
run() { echo "$*" >> "$OUT/progress.log"; timeout -k 10 150 env "$@" >> "$J" 2>> "$OUT/err.log" || { echo "FAILED: $*" >> "$OUT/err.log"; return 1; }; }
B="python bench.py --steps 10 --warmup 2 --verify 60 --no-phase-step"
for rep in 1 2 3; do
  for sz in "--height 4096" "--height 4096 --rehearse-rccl" "--height 8192 --rehearse-rccl" "--size 8192" "--size 32768"; do
    run GOL_AB=default $B $sz || exit 1
    run GOL_AB=nolink GOL_LINK=0 $B $sz || exit 1
  done
done
