#!/bin/bash
# Resident epochs: compute-phase time and shader clock between refreshes,
# exact vs probe (no exchange), on a fresh random grid and after warmup.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/res3
mkdir -p $O
for mode in exact probe; do
  pr=0; [ $mode = probe ] && pr=1
  for when in fresh warm; do
    if [ $when = fresh ]; then at=0; args="--prewarm 0 --warmup 0 --steps 1 --gens-per-step 128"; else at=40; args="--prewarm 0 --warmup 3 --steps 3"; fi
    GOL_RESIDENT=1 GOL_RES_PROBE=$pr GOL_RES_TRACE=$at:$O/trace_${mode}_${when}.csv timeout -k 10 120 python bench.py --height 4096 $args --verify 0 --no-phase-step > $O/${mode}_${when}.json 2>> $O/err.log
    rc=$?; echo "$mode $when rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python scripts/res_trace.py $O/trace_${mode}_${when}.csv | tail -1
  done
done
