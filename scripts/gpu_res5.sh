#!/bin/bash
# Resident epochs, barrier vs LDS-counter hand-off: totals and a kernel trace.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/res5
mkdir -p $O
T=$O/tiles.jsonl; : > $T
run() {  # label, env..., -- bench args
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 150 python bench.py --steps 10 --warmup 2 --no-phase-step "$@" > $O/one.json 2>> $O/bench.err
  local rc=$?
  echo "{\"label\": \"$label\", \"rc\": $rc, \"run\": $(cat $O/one.json 2>/dev/null || echo null)}" >> $T
  echo "$label rc=$rc $(python3 -c "import json,sys; d=json.load(open('$O/one.json')); print(round(d['ms_per_step'],3), 'ms', d['verified'], d['config']['kernel'], d['config']['epoch'], d['config']['step_stop_reasons'])" 2>/dev/null)"
  return $rc
}
S=alt_so/sync1/_gol.so
for H in 4096 8192; do
  run "h$H default" GOL_RESIDENT=0 -- --height $H || exit $?
  run "h$H resident" GOL_RESIDENT=1 -- --height $H || exit $?
  run "h$H resident sync1" GOL_NATIVE_SO=$S GOL_RESIDENT=1 -- --height $H || exit $?
  run "h$H resident sync1 D256" GOL_NATIVE_SO=$S GOL_RESIDENT=1 GOL_RES_D=256 -- --height $H || exit $?
  GOL_NATIVE_SO=$S GOL_RESIDENT=1 GOL_RES_TRACE=20:$O/trace_h$H.csv timeout -k 10 120 python bench.py --height $H --prewarm 0 --warmup 3 --steps 2 --verify 0 --no-phase-step > $O/tr.json 2>> $O/err.log
  rc=$?; echo "trace h$H rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python scripts/res_trace.py $O/trace_h$H.csv | head -6; python scripts/res_trace.py $O/trace_h$H.csv | tail -1
done
