#!/bin/bash
# Packed LDS tile: row-major tile order (default) vs XCD-aware (GOL_LDS_XCD=1), and 16 waves per workgroup.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/lds7
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -k "lds" -q --timeout 120 --timeout-method thread > $O/pytest_lds_xcd.log 2>&1
rc=$?; echo "lds tests rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest_lds_xcd.log | tail -8; [ $rc -eq 0 ] || exit $rc
T=$O/lds.jsonl; : > $T
for S in 8192 32768; do
  st=20; [ $S = 32768 ] && st=3
  for v in default xcd waves16 default xcd waves16; do
    so=""; x=0; [ $v = waves16 ] && so=alt_so/$v/_gol.so; [ $v = xcd ] && x=1
    GOL_LDS_XCD=$x GOL_NATIVE_SO=$so GOL_U8_KERNEL=lds timeout -k 10 200 python bench.py --layout u8 --u8-compute bytes --no-phase-step --size $S --steps $st --warmup 1 > $O/one.json 2>> $O/err.log
    rc=$?; echo "{\"label\": \"$v $S\", \"rc\": $rc, \"run\": $(cat $O/one.json 2>/dev/null || echo null)}" >> $T
    echo "$v $S rc=$rc $(python3 -c "import json; d=json.load(open('$O/one.json')); us=d['ms_per_step']*1e3/d['config']['gens_per_step']; print(round(us,2), 'us/gen', '%.3g'%d['value'], d['verified'])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
