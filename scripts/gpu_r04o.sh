#!/bin/bash
# Round 4 batch o: VALU issue cost by instruction form and operand banks.
set -o pipefail
OUT=gpurun_out/${1:-r04o}
mkdir -p "$OUT"
timeout -k 10 120 ./bin/ubench_vop3 2048 > "$OUT/ubench_vop3.txt" 2>&1
