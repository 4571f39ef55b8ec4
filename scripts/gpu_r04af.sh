#!/bin/bash
# Round 4 batch af: 65536^2 (BASELINE config 4's grid) verified on light-cone
# row bands (bench.py ORACLE_WHOLE_CELLS), after the whole-grid fp32 oracle
# faulted the GPU at 2^32 elements.
set -o pipefail
OUT=gpurun_out/${1:-r04af}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 400 python bench.py --size 65536 --steps 3 --warmup 1 --verify 30 > "$OUT/bench_65536.json" 2> "$OUT/bench_65536.err"
