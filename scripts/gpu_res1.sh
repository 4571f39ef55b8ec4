#!/bin/bash
# Resident epochs: GPU tests, then the rank tiles against the default kernels.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/res1
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -k resident -v --timeout 120 --timeout-method thread > $O/pytest_resident.log 2>&1
rc=$?; echo "resident tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $O/pytest_resident.log | tail -8; [ $rc -eq 0 ] || exit $rc
GOL_NATIVE_SO=alt_so/sync1/_gol.so timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -k resident -v --timeout 120 --timeout-method thread > $O/pytest_resident_sync1.log 2>&1
rc=$?; echo "resident tests (sync1) rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $O/pytest_resident_sync1.log | tail -8; [ $rc -eq 0 ] || exit $rc
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
  run "h$H resident k8" GOL_RESIDENT=1 GOL_RES_K=8 -- --height $H || exit $?
  run "h$H resident k8 sync1" GOL_NATIVE_SO=alt_so/sync1/_gol.so GOL_RESIDENT=1 GOL_RES_K=8 -- --height $H || exit $?
  run "h$H resident k8 sync1 probe" GOL_NATIVE_SO=alt_so/sync1/_gol.so GOL_RESIDENT=1 GOL_RES_K=8 GOL_RES_PROBE=1 -- --height $H --verify 0 || exit $?
  run "h$H resident k16" GOL_RESIDENT=1 GOL_RES_K=16 -- --height $H || exit $?
  run "h$H resident k8 probe" GOL_RESIDENT=1 GOL_RES_K=8 GOL_RES_PROBE=1 -- --height $H --verify 0 || exit $?
  run "h$H rehearse default" GOL_RESIDENT=0 -- --height $H --rehearse-rccl || exit $?
  run "h$H rehearse resident k8 D256" GOL_RESIDENT=1 GOL_RES_K=8 -- --height $H --rehearse-rccl || exit $?
  run "h$H rehearse resident k8 D128" GOL_RESIDENT=1 GOL_RES_K=8 GOL_RES_D=128 -- --height $H --rehearse-rccl || exit $?
done
run "h16384 default" GOL_RESIDENT=0 -- --height 16384 || exit $?
run "h16384 resident k8" GOL_RESIDENT=1 GOL_RES_K=8 -- --height 16384 || exit $?
run "h16384 rehearse resident k8" GOL_RESIDENT=1 GOL_RES_K=8 -- --height 16384 --rehearse-rccl || exit $?
