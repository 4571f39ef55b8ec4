#!/bin/bash
# Linked launches: exactness, then the 8-GPU rank tile with and without.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/link
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -q -x -k "linked" --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -15 $O/pytest.log; echo "tests rc=$rc"; [ $rc -le 1 ] || exit $rc; [ $rc -eq 0 ] || exit 1
: > $O/bench.jsonl; : > $O/labels.txt
for i in 1 2 3; do
  for link in 0 1; do
    timeout -k 10 200 env GOL_LINK=$link python bench.py --height 4096 --verify 100 --no-phase-step >> $O/bench.jsonl 2>> $O/bench.err || exit $?
    echo "tile link=$link" >> $O/labels.txt
  done
done
for link in 0 1; do
  timeout -k 10 200 env GOL_LINK=$link python bench.py --height 8192 --verify 0 --no-phase-step >> $O/bench.jsonl 2>> $O/bench.err || exit $?
  echo "4gpu-tile link=$link" >> $O/labels.txt
  timeout -k 10 200 env GOL_LINK=$link python bench.py --height 4096 --rehearse-rccl --verify 0 --no-phase-step >> $O/bench.jsonl 2>> $O/bench.err || exit $?
  echo "tile-rccl link=$link" >> $O/labels.txt
done
python3 - <<'PY'
import json
labels = [l.strip() for l in open("gpurun_out/link/labels.txt")]
for lab, l in zip(labels, open("gpurun_out/link/bench.jsonl")):
    d = json.loads(l); c = d["config"]
    print("%-16s %-12s T=%-2d %8.3f ms/step %.4g verified=%s" % (lab, c["grid"], c["tmax"], d["ms_per_step"], d["value"], d["verified"]))
PY
