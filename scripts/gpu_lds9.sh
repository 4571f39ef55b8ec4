#!/bin/bash
# Packed LDS tile at 8192^2 with 16-wave workgroups: 160 rows (default) vs 128 / 192.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/lds9
mkdir -p $O
T=$O/lds.jsonl; : > $T
for v in default r128 r192 default r128 r192; do
  so=""; [ $v != default ] && so=alt_so/$v/_gol.so
  GOL_NATIVE_SO=$so GOL_U8_KERNEL=lds timeout -k 10 200 python bench.py --layout u8 --u8-compute bytes --no-phase-step --size 8192 --steps 20 --warmup 1 > $O/one.json 2>> $O/err.log
  rc=$?; echo "{\"label\": \"$v 8192\", \"rc\": $rc, \"run\": $(cat $O/one.json 2>/dev/null || echo null)}" >> $T
  echo "$v rc=$rc $(python3 -c "import json; d=json.load(open('$O/one.json')); us=d['ms_per_step']*1e3/d['config']['gens_per_step']; print(round(us,2), 'us/gen', '%.3g'%d['value'], d['verified'])")"
  [ $rc -eq 0 ] || exit $rc
done
