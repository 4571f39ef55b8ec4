#!/bin/bash
# Round 4 batch e: 8-GPU rank tile (32768 x 4096) kernel variants with the
# round-4 defaults (4-wave groups at T <= 8, chained-group acquire), and the
# per-rank tiles of N = 2 / 4 with the one-rank RCCL rehearsal.
set -o pipefail
OUT=gpurun_out/${1:-r04e}
mkdir -p "$OUT"
timeout -k 10 120 bin/ubench_vbody 3000 > "$OUT/ubench_vbody.txt" 2>&1 || exit $?
J="$OUT/tile.jsonl"; : > "$J"
run() { timeout -k 10 120 env "$@" >> "$J" 2>> "$OUT/err.log" || { echo "FAILED: $*" >> "$OUT/err.log"; return 1; }; }
B="python bench.py --steps 10 --warmup 2 --verify 0 --no-phase-step"
for rep in 1 2 3; do
  run GOL_XLANE=-1 $B --height 4096 || exit 1
  run GOL_XLANE=3 $B --height 4096 --tmax 8 || exit 1
  run GOL_XLANE=0 $B --height 4096 --tmax 8 || exit 1
  run GOL_XLANE=3 GOL_GROUP_SMALL=8 $B --height 4096 --tmax 8 || exit 1
  run GOL_XLANE=3 $B --height 4096 --tmax 12 || exit 1
  run GOL_XLANE=0 $B --height 4096 --tmax 12 || exit 1
  run GOL_XLANE=-1 GOL_GROUP=4 $B --height 4096 || exit 1
done
for rep in 1 2; do
  for h in 16384 8192 4096; do
    run GOL_XLANE=-1 $B --height $h --rehearse-rccl || exit 1
  done
done
