#!/bin/bash
# Round 4 batch i: level-body microbenchmark with the two-word adder window,
# then the PMC occupancy passes (batch h).
set -o pipefail
OUT=gpurun_out/${1:-r04i}
mkdir -p "$OUT"
timeout -k 10 180 bin/ubench_vbody 3000 > "$OUT/ubench_vbody.txt" 2>&1 || exit $?
bash scripts/gpu_r04h.sh r04i_pmc || exit $?
