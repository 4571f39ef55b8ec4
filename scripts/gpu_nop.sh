#!/bin/bash
# Adder window without the trailing s_nop inside its asm block (the compiler
# pads the hazard after the block itself): exactness, then A/B on the
# headline grid and the 2- / 4-GPU rank tiles, interleaved.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/nop
mkdir -p $O
GOL_NATIVE_SO=alt_so/nonop/_gol.so timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -k "adder or every_temporal or row_strips" -q --timeout 120 --timeout-method thread > $O/pytest_nonop.log 2>&1
rc=$?; echo "adder tests (no nop) rc=$rc"; tail -2 $O/pytest_nonop.log; [ $rc -eq 0 ] || exit $rc
T=$O/ab.jsonl; : > $T
for rep in 1 2; do
  for v in default nonop; do
    so=""; [ $v != default ] && so=alt_so/$v/_gol.so
    for H in 32768 16384 8192; do
      GOL_NATIVE_SO=$so timeout -k 10 200 python bench.py --height $H --steps 20 --warmup 5 --no-phase-step --verify 0 > $O/one.json 2>> $O/err.log
      rc=$?; echo "{\"label\": \"$v h$H rep$rep\", \"rc\": $rc, \"run\": $(cat $O/one.json 2>/dev/null || echo null)}" >> $T
      echo "$v h$H rep$rep rc=$rc $(python3 -c "import json; d=json.load(open('$O/one.json')); print(round(d['ms_per_step'],3), 'ms', d['config']['kernel'])")"
      [ $rc -eq 0 ] || exit $rc
    done
  done
done
