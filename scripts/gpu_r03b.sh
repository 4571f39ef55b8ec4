#!/bin/bash
# Round 3 GPU pass b: T = 48 byte-pass tests, byte-layout bench A/B (T = 48
# pipelined pairs vs T = 32 grouped) on 32768^2, 65536^2 and the 8-GPU 1M^2
# per-rank share, then the occupancy / LDS PMC passes.  Every step has its
# own limit; a step that times out or faults ends the script.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03b
mkdir -p $O
step() {
  local name=$1 limit=$2
  shift 2
  timeout -k 10 "$limit" "$@"
  local rc=$?
  echo "step $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop"; exit $rc; fi
  return 0
}
step t48 300 python -u -m pytest tests/test_gpu.py -q -k "t48 or deep_byte" --timeout 240 --timeout-method thread > $O/pytest_t48.log 2>&1
tail -2 $O/pytest_t48.log
: > $O/u8.jsonl
for args in "--layout u8" "--layout u8 --tmax 32" "--layout u8 --size 65536 --steps 3" "--layout u8 --size 65536 --steps 3 --tmax 32" \
            "--layout u8 --size 8192" "--layout u8 --size 32768 --height 16384" "--layout u8 --size 32768 --height 16384 --tmax 32"; do
  step "u8 $args" 200 python bench.py --steps 5 --warmup 1 --verify 0 --no-phase-step $args >> $O/u8.jsonl 2>> $O/u8.err
done
for args in "" "--tmax 32"; do
  step "u8 1M share $args" 300 python bench.py --layout u8 --size 1048576 --height 131072 --gens-per-step 96 --steps 2 --warmup 1 --prewarm 0 --verify 0 --no-phase-step $args >> $O/u8.jsonl 2>> $O/u8.err
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r03b/u8.jsonl"):
    d = json.loads(l); c = d["config"]
    print("%-16s T=%-2d ep=%-4d %8.3f ms/step %.4g" % (c["grid"], c["tmax"], c["epoch"], d["ms_per_step"], d["value"]))
PY
bash scripts/gpu_pmc_r03.sh
