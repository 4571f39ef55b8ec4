#!/bin/bash
# Multi-generation LDS-tiled byte kernel: exactness, then T = 1 / 2 / 4 / 8.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/lds2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -k "lds" -q --timeout 120 --timeout-method thread > $O/pytest_lds.log 2>&1
rc=$?; echo "lds tests rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest_lds.log | tail -8; [ $rc -eq 0 ] || exit $rc
GOL_LDS_ADD=1 timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -k "lds" -q --timeout 120 --timeout-method thread > $O/pytest_lds_add.log 2>&1
rc=$?; echo "lds tests (adder) rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest_lds_add.log | tail -8; [ $rc -eq 0 ] || exit $rc
T=$O/lds.jsonl; : > $T
run() {
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py --layout u8 --u8-compute bytes --no-phase-step "$@" > $O/one.json 2>> $O/err.log
  local rc=$?
  echo "{\"label\": \"$label\", \"rc\": $rc, \"run\": $(cat $O/one.json 2>/dev/null || echo null)}" >> $T
  echo "$label rc=$rc $(python3 -c "import json; d=json.load(open('$O/one.json')); g=d['config']['grid']; n=int(g.split('x')[0])*int(g.split('x')[1]); us=d['ms_per_step']*1e3/d['config']['gens_per_step']; print(round(us,2), 'us/gen', '%.3g'%d['value'], d['verified'], d['config']['tmax'], d['config']['epoch'])")"
  return $rc
}
for S in 8192 32768; do
  st=20; [ $S = 32768 ] && st=3
  for t in 8; do
    run "lds bytes T$t $S" GOL_U8_KERNEL=lds GOL_LDS_PACK=0 GOL_LDS_T=$t -- --size $S --steps $st --warmup 1 || exit $?
  done
  for t in 16 32; do
    run "lds packed T$t $S" GOL_U8_KERNEL=lds GOL_LDS_PACK=1 GOL_LDS_T=$t -- --size $S --steps $st --warmup 1 || exit $?
    run "lds packed adder T$t $S" GOL_U8_KERNEL=lds GOL_LDS_ADD=1 GOL_LDS_PACK=1 GOL_LDS_T=$t -- --size $S --steps $st --warmup 1 || exit $?
  done
done
