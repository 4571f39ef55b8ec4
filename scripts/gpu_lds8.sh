#!/bin/bash
# Packed LDS tile: 8 / 16 waves per workgroup chosen by grid size (auto) vs forced, three sizes.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/lds8
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -k "lds" -q --timeout 120 --timeout-method thread > $O/pytest_lds_waves.log 2>&1
rc=$?; echo "lds tests rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest_lds_waves.log | tail -8; [ $rc -eq 0 ] || exit $rc
T=$O/lds.jsonl; : > $T
for S in 8192 16384 32768; do
  st=20; [ $S = 16384 ] && st=8; [ $S = 32768 ] && st=3
  for v in 0 8 16 0; do
    GOL_LDS_WAVES=$v GOL_U8_KERNEL=lds timeout -k 10 200 python bench.py --layout u8 --u8-compute bytes --no-phase-step --size $S --steps $st --warmup 1 > $O/one.json 2>> $O/err.log
    rc=$?; echo "{\"label\": \"waves=$v $S\", \"rc\": $rc, \"run\": $(cat $O/one.json 2>/dev/null || echo null)}" >> $T
    echo "waves=$v $S rc=$rc $(python3 -c "import json; d=json.load(open('$O/one.json')); us=d['ms_per_step']*1e3/d['config']['gens_per_step']; print(round(us,2), 'us/gen', '%.3g'%d['value'], d['verified'])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
