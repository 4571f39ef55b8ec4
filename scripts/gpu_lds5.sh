#!/bin/bash
# Packed LDS tile: LDS rows 128 (default) / 160 / 192 at T = 32.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/lds5
mkdir -p $O
T=$O/lds.jsonl; : > $T
for S in 8192 32768; do
  st=20; [ $S = 32768 ] && st=3
  for v in default rows160 rows192 default rows160 rows192; do
    so=""; [ $v != default ] && so=alt_so/$v/_gol.so
    GOL_NATIVE_SO=$so GOL_U8_KERNEL=lds timeout -k 10 200 python bench.py --layout u8 --u8-compute bytes --no-phase-step --size $S --steps $st --warmup 1 > $O/one.json 2>> $O/err.log
    rc=$?; echo "{\"label\": \"$v $S\", \"rc\": $rc, \"run\": $(cat $O/one.json 2>/dev/null || echo null)}" >> $T
    echo "$v $S rc=$rc $(python3 -c "import json; d=json.load(open('$O/one.json')); us=d['ms_per_step']*1e3/d['config']['gens_per_step']; print(round(us,2), 'us/gen', '%.3g'%d['value'], d['verified'])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
# 8-GPU rank tile shapes: 1x8 strip (32768 x 4096) vs 2x4 block (16384 x 8192), wrap and halo columns.
for spec in "strip:--size 32768 --height 4096" "block:--size 16384 --height 8192"; do
  for wr in 1 0; do
    name=${spec%%:*}; args=${spec#*:}
    GOL_WRAP=$wr timeout -k 10 200 python bench.py $args --steps 20 --warmup 3 > $O/one.json 2>> $O/err.log
    rc=$?; echo "{\"label\": \"$name wrap=$wr\", \"rc\": $rc, \"run\": $(cat $O/one.json 2>/dev/null || echo null)}" >> $O/tiles.jsonl
    echo "$name wrap=$wr rc=$rc $(python3 -c "import json; d=json.load(open('$O/one.json')); print(d['ms_per_step'], 'ms', '%.3g'%d['value'], d['verified'], d['config'].get('kernel','')[:80])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
