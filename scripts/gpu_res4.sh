#!/bin/bash
# Resident kernel body variants: compute time between refreshes (8-GPU tile, warm).
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/res4
mkdir -p $O
for v in default rf0 rf4 sync1 sync1rf0; do
  so=""; [ $v != default ] && so=alt_so/$v/_gol.so
  GOL_NATIVE_SO=$so GOL_RESIDENT=1 GOL_RES_TRACE=40:$O/trace_$v.csv timeout -k 10 120 python bench.py --height 4096 --prewarm 0 --warmup 3 --steps 5 --verify 0 --no-phase-step > $O/$v.json 2>> $O/err.log
  rc=$?; echo "$v rc=$rc $(python3 -c "import json; d=json.load(open('$O/$v.json')); print(round(d['ms_per_step'],3), 'ms/1000 gens', d['config']['step_stop_reasons'])")"; [ $rc -eq 0 ] || exit $rc
  python scripts/res_trace.py $O/trace_$v.csv | tail -1
done
