#!/bin/bash
# Round 4 batch ah: per-wave traces of two consecutive launches, linked
# (default) and not (GOL_LINK=0), on 8192^2 and the 8-GPU rank tile
# (multi-rank schedule): scripts/wg_trace.py --pair.
set -o pipefail
OUT=gpurun_out/${1:-r04ah}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
B="python bench.py --steps 2 --warmup 1 --verify 0 --no-phase-step --prewarm 0"
timeout -k 10 120 env GOL_WG_TRACE="301:$OUT/pair_8192_linked.csv:pair" $B --size 8192 > "$OUT/b1.json" 2> "$OUT/err.log" || exit $?
timeout -k 10 120 env GOL_LINK=0 GOL_WG_TRACE="301:$OUT/pair_8192_plain.csv:pair" $B --size 8192 > "$OUT/b2.json" 2>> "$OUT/err.log" || exit $?
timeout -k 10 120 env GOL_WG_TRACE="101:$OUT/pair_tile_linked.csv:pair" $B --height 4096 --rehearse-rccl > "$OUT/b3.json" 2>> "$OUT/err.log" || exit $?
timeout -k 10 120 env GOL_LINK=0 GOL_WG_TRACE="101:$OUT/pair_tile_plain.csv:pair" $B --height 4096 --rehearse-rccl > "$OUT/b4.json" 2>> "$OUT/err.log"
