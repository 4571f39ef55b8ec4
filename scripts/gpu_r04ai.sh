#!/bin/bash
# Round 4 batch ai: is the 8192^2 loop host-bound?  Same launch count, less
# work per launch (8192 x 4096 / x 2048), and a HIP runtime trace of the
# 8192^2 run (host API timestamps; no counters).
set -o pipefail
OUT=gpurun_out/${1:-r04ai}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
J="$OUT/ab.jsonl"; : > "$J"
run() { echo "$*" >> "$OUT/progress.log"; timeout -k 10 150 env "$@" >> "$J" 2>> "$OUT/err.log" || { echo "FAILED: $*" >> "$OUT/err.log"; return 1; }; }
B="python bench.py --steps 10 --warmup 2 --verify 0 --no-phase-step --size 8192"
for rep in 1 2; do
  for h in 8192 4096 2048; do
    run GOL_AB=h$h $B --height $h --tmax 8 || exit 1
    run GOL_AB=h$h GOL_LINK=1 $B --height $h --tmax 8 || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --runtime-trace -d $OUT/rt -o run -- python3 bench.py --steps 3 --warmup 1 --verify 0 --no-phase-step --size 8192 > $OUT/rt.json 2> $OUT/rt.err
