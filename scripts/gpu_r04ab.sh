#!/bin/bash
# Round 4 batch ab: price of the adder window's cross-lane carries inside the
# level body (timing probe with the carries removed, wrong cells).
set -o pipefail
OUT=gpurun_out/${1:-r04ab}
mkdir -p "$OUT"
timeout -k 10 120 ./bin/ubench_vbody > "$OUT/vbody_carry.txt" 2>&1 || exit $?
timeout -k 10 120 ./bin/ubench_vbody_fake > "$OUT/vbody_fake.txt" 2>&1
