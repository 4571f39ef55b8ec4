#!/bin/bash
# Round 4 batch f: step-boundary trim A/B (compare with r04d/r04e), the
# multi-rank epoch depth on the 8-GPU rank tile (one-rank RCCL rehearsal),
# and kernel traces of the headline, 8192^2 u8 and the rehearsed 8-GPU tile.
set -o pipefail
OUT=gpurun_out/${1:-r04f}
mkdir -p "$OUT"
J="$OUT/ab.jsonl"; : > "$J"
run() { timeout -k 10 120 env "$@" >> "$J" 2>> "$OUT/err.log" || { echo "FAILED: $*" >> "$OUT/err.log"; return 1; }; }
B="python bench.py --steps 10 --warmup 2 --verify 0 --no-phase-step"
for rep in 1 2 3; do
  run GOL_X=0 $B --size 8192 || exit 1
  run GOL_X=0 $B --size 8192 --layout u8 || exit 1
  run GOL_X=0 $B --height 4096 || exit 1
  run GOL_X=0 $B || exit 1
done
for rep in 1 2; do
  for e in 128 192 256 384; do
    run GOL_X=0 $B --height 4096 --rehearse-rccl --epoch $e || exit 1
  done
done
export TMPDIR=/tmp
P="--steps 5 --warmup 1 --verify 0 --no-phase-step"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/prof_32768" -o run -- python3 bench.py $P > "$OUT/prof_32768.log" 2>&1 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/prof_8192_u8" -o run -- python3 bench.py $P --size 8192 --layout u8 > "$OUT/prof_8192_u8.log" 2>&1 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/prof_tile_rehearsal" -o run -- python3 bench.py $P --height 4096 --rehearse-rccl > "$OUT/prof_tile.log" 2>&1 || exit 1
# The experimental build (variants measured slower, compiled out of the default
# module) still exact: its GPU tests against the alternate module.
GOL_NATIVE_SO=exp_so/_gol.so timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  -m "gpu and experimental" tests/test_gpu.py > "$OUT/experimental_tier.log" 2>&1 || exit $?
