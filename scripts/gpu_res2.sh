#!/bin/bash
# Resident epochs: GPU tests, refresh phase traces and the rank tiles.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/res2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -k resident -v --timeout 120 --timeout-method thread > $O/pytest_resident.log 2>&1
rc=$?; echo "resident tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $O/pytest_resident.log | tail -8; [ $rc -eq 0 ] || exit $rc
for H in 4096 8192; do
  GOL_RESIDENT=1 GOL_RES_TRACE=6:$O/trace_h$H.csv timeout -k 10 120 python bench.py --height $H --steps 3 --warmup 1 --prewarm 0 --verify 0 --no-phase-step > $O/h$H.json 2>> $O/err.log
  rc=$?; echo "trace h$H rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python scripts/res_trace.py $O/trace_h$H.csv | head -14
done
T=$O/tiles.jsonl; : > $T
run() {  # label, env..., -- bench args
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 150 python bench.py --steps 10 --warmup 2 --no-phase-step "$@" > $O/one.json 2>> $O/bench.err
  local rc=$?
  echo "{\"label\": \"$label\", \"rc\": $rc, \"run\": $(cat $O/one.json 2>/dev/null || echo null)}" >> $T
  echo "$label rc=$rc $(python3 -c "import json,sys; d=json.load(open('$O/one.json')); print(round(d['ms_per_step'],3), 'ms', d['verified'], d['config']['kernel'], d['config']['epoch'])" 2>/dev/null)"
  return $rc
}
for H in 4096 8192; do
  run "h$H default" GOL_RESIDENT=0 -- --height $H || exit $?
  run "h$H resident" GOL_RESIDENT=1 -- --height $H || exit $?
  run "h$H resident k8" GOL_RESIDENT=1 GOL_RES_K=8 -- --height $H || exit $?
  run "h$H rehearse default" GOL_RESIDENT=0 -- --height $H --rehearse-rccl || exit $?
  run "h$H rehearse resident" GOL_RESIDENT=1 -- --height $H --rehearse-rccl || exit $?
done
run "h16384 default" GOL_RESIDENT=0 -- --height 16384 || exit $?
run "h16384 resident" GOL_RESIDENT=1 -- --height 16384 || exit $?
