#!/bin/bash
# LDS-tiled single-step byte kernel (BASELINE config 2): tile heights, vs the
# T = 1 register kernel, 8192^2 and 32768^2.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/lds
mkdir -p $O
T=$O/lds.jsonl; : > $T
run() {
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py --layout u8 --u8-compute bytes --no-phase-step "$@" > $O/one.json 2>> $O/err.log
  local rc=$?
  echo "{\"label\": \"$label\", \"rc\": $rc, \"run\": $(cat $O/one.json 2>/dev/null || echo null)}" >> $T
  echo "$label rc=$rc $(python3 -c "import json; d=json.load(open('$O/one.json')); g=d['config']['grid']; n=int(g.split('x')[0])*int(g.split('x')[1]); us=d['ms_per_step']*1e3/d['config']['gens_per_step']; print(round(us,2), 'us/gen', '%.3g'%d['value'], round(2*n/us/1e6,2), 'TB/s', d['verified'])")"
  return $rc
}
for S in 8192 32768; do
  st=20; [ $S = 32768 ] && st=2
  run "lds32 $S" GOL_U8_KERNEL=lds GOL_LDS_ROWS=32 -- --size $S --steps $st --warmup 1 || exit $?
  run "lds64 $S" GOL_U8_KERNEL=lds GOL_LDS_ROWS=64 -- --size $S --steps $st --warmup 1 || exit $?
  run "reg T1 $S" -- --size $S --tmax 1 --steps $st --warmup 1 || exit $?
done
