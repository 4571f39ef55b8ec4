#!/bin/bash
# A/B on one box, alternating: chain autotune vs off on the headline; byte
# layout DPP vs carry window at T = 48 / 32.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/ab
mkdir -p $O
: > $O/ab.jsonl
run() {  # run LABEL ENV... -- ARGS
  local label=$1; shift
  timeout -k 10 200 env "$@" >> $O/ab.jsonl 2>> $O/ab.err
  local rc=$?
  [ $rc -eq 0 ] || { echo "$label rc=$rc"; exit $rc; }
  echo "$label" >> $O/labels.txt
}
: > $O/labels.txt
for i in 1 2 3; do
  run chain_auto GOL_CHAIN=-1 python bench.py --verify 0 --no-phase-step
  run chain_off GOL_CHAIN=0 python bench.py --verify 0 --no-phase-step
done
for i in 1 2; do
  run u8_dpp GOL_XLANE=0 python bench.py --layout u8 --steps 5 --warmup 1 --verify 0 --no-phase-step
  run u8_carry GOL_XLANE=2 python bench.py --layout u8 --steps 5 --warmup 1 --verify 0 --no-phase-step
  run u8_carry_t32 GOL_XLANE=2 python bench.py --layout u8 --tmax 32 --steps 5 --warmup 1 --verify 0 --no-phase-step
done
python3 - <<'PY'
import json
labels = [l.strip() for l in open("gpurun_out/ab/labels.txt")]
for lab, l in zip(labels, open("gpurun_out/ab/ab.jsonl")):
    d = json.loads(l); c = d["config"]
    print("%-14s %-12s T=%-2d %8.3f ms/step %.4g" % (lab, c["grid"], c["tmax"], d["ms_per_step"], d["value"]))
PY
