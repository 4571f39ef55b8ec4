#!/bin/bash
# Byte layout: epochs on bit words (u8_compute bits, the GPU default) vs the
# byte kernels (bytes), on the BASELINE byte-layout shapes.  One JSON line per run.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/u8bits
mkdir -p $O
: > $O/runs.jsonl
step() {  # label, timeout, command...
  local label=$1 t=$2; shift 2
  echo "== $label" >&2
  timeout -k 10 $t "$@" > $O/one.json 2>> $O/err.log
  local rc=$?
  echo "{\"label\": \"$label\", \"rc\": $rc, \"run\": $(cat $O/one.json 2>/dev/null || echo null)}" >> $O/runs.jsonl
  echo "$label rc=$rc $(cut -c1-200 $O/one.json)" >&2
  return $rc
}
for m in bits bytes; do
  step "32768 u8 $m" 300 python bench.py --layout u8 --u8-compute $m --steps 10 --warmup 3 || exit $?
done
for m in bits bytes; do
  step "8192 u8 $m" 300 python bench.py --layout u8 --u8-compute $m --size 8192 --steps 20 --warmup 5 || exit $?
done
for m in bits bytes; do
  step "1M share u8 $m" 400 python bench.py --layout u8 --u8-compute $m --size 1048576 --height 131072 \
    --gens-per-step 384 --steps 2 --warmup 1 --prewarm 0 --verify 0 --no-phase-step || exit $?
done
