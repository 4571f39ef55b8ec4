#!/bin/bash
# Per-run pack of the byte layout on bit words: GPU tier, u8 measurements, kernel traces.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03e
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "gpu tier rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest_gpu.log | tail -30; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_u8bits.sh || exit $?
bash scripts/gpu_trace_r03.sh
# 8-GPU rank tile: temporal depth / window sweep (tile alone, one GPU)
T=gpurun_out/r03e/tile_sweep.jsonl; : > $T
for spec in "def:" "t8:--tmax 8" "t12:--tmax 12" "t8add:--tmax 8 XL=3" "t8dpp:--tmax 8 XL=0" "t12dpp:--tmax 12 XL=0"; do
  name=${spec%%:*}; args=${spec#*:}; xl=-1
  case "$args" in *XL=*) xl=${args##*XL=}; args=${args%XL=*};; esac
  GOL_XLANE=$xl timeout -k 10 200 python bench.py --height 4096 --steps 20 --warmup 5 --verify 0 --no-phase-step $args > $O/one.json 2>> $O/tile.err
  rc=$?; echo "{\"label\": \"$name\", \"rc\": $rc, \"run\": $(cat $O/one.json 2>/dev/null || echo null)}" >> $T
  echo "tile $name rc=$rc $(cut -c1-150 $O/one.json)"; [ $rc -eq 0 ] || exit $rc
done
