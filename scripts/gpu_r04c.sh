#!/bin/bash
# Round 4 batch c: the N = 8 bench rehearsal at the headline grid, 8192^2
# with the small-tile T choice, the chained-group acquire's cost on the 8-GPU
# rank tile, and a kernel trace of 8192^2.
set -o pipefail
OUT=gpurun_out/${1:-r04c}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python bench.py --gpus 8 --share-gpus --steps 2 --warmup 1 --prewarm 0 --verify 240 \
  > "$OUT/bench8_shared.json" 2> "$OUT/bench8_shared.err" || exit $?
J="$OUT/ab.jsonl"; : > "$J"
run() { timeout -k 10 120 env "$@" >> "$J" 2>> "$OUT/err.log" || { echo "FAILED: $*" >> "$OUT/err.log"; return 1; }; }
B="python bench.py --steps 10 --warmup 2 --verify 0 --no-phase-step"
for rep in 1 2 3; do
  run GOL_CHAIN_ACQUIRE=1 $B --height 4096 || exit 1
  run GOL_CHAIN_ACQUIRE=0 $B --height 4096 || exit 1
done
for rep in 1 2; do
  run GOL_CHAIN_ACQUIRE=1 $B --size 8192 || exit 1
  run GOL_CHAIN_ACQUIRE=1 $B --size 8192 --layout u8 || exit 1
  run GOL_GROUP=4 $B --size 8192 || exit 1
  run GOL_GROUP=-1 $B --size 8192 || exit 1
  run GOL_CHAIN=0 $B --size 8192 || exit 1
  run GOL_CHAIN=1 $B --size 8192 || exit 1
  run GOL_CHAIN_ACQUIRE=0 $B --size 8192 || exit 1
done
timeout -k 10 120 python bench.py --size 8192 --steps 10 --warmup 2 > "$OUT/bench8192_verified.json" 2>> "$OUT/err.log" || exit 1
timeout -k 10 120 python bench.py --size 8192 --layout u8 --steps 10 --warmup 2 > "$OUT/bench8192_u8_verified.json" 2>> "$OUT/err.log" || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/prof8192" -o run -- python3 bench.py --size 8192 --steps 5 --warmup 1 --verify 0 --no-phase-step > "$OUT/prof8192.log" 2>&1 || exit 1
