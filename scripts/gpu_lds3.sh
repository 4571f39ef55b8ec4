#!/bin/bash
# Packed LDS tile height: 64 / 128 (default) / 256 rows, T = 16 and 32.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/lds3
mkdir -p $O
T=$O/lds.jsonl; : > $T
for S in 8192 32768; do
  st=20; [ $S = 32768 ] && st=3
  for v in rows64 default rows256; do
    so=""; [ $v != default ] && so=alt_so/$v/_gol.so
    for t in 16 32; do
      [ $v = rows64 ] && [ $t = 32 ] && continue
      GOL_NATIVE_SO=$so GOL_U8_KERNEL=lds GOL_LDS_T=$t timeout -k 10 200 python bench.py --layout u8 --u8-compute bytes --no-phase-step --size $S --steps $st --warmup 1 > $O/one.json 2>> $O/err.log
      rc=$?; echo "{\"label\": \"$v T$t $S\", \"rc\": $rc, \"run\": $(cat $O/one.json 2>/dev/null || echo null)}" >> $T
      echo "$v T$t $S rc=$rc $(python3 -c "import json; d=json.load(open('$O/one.json')); us=d['ms_per_step']*1e3/d['config']['gens_per_step']; print(round(us,2), 'us/gen', '%.3g'%d['value'], d['verified'])")"
      [ $rc -eq 0 ] || exit $rc
    done
  done
done
