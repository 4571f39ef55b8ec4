#!/bin/bash
# Round 4 batch ac: level-body rate against resident waves per SIMD (1-8).
set -o pipefail
OUT=gpurun_out/${1:-r04ac}
mkdir -p "$OUT"
timeout -k 10 120 ./bin/ubench_vbody 3000 1 > "$OUT/vbody_occupancy.txt" 2>&1
