#!/bin/bash
# Round 4 batch ak: host cost of launch patterns (csrc/tools/ubench_launch.hip).
set -o pipefail
OUT=gpurun_out/${1:-r04ak}
mkdir -p "$OUT"
timeout -k 10 120 ./bin/ubench_launch 2000 > "$OUT/ubench_launch.txt" 2>&1
