#!/bin/bash
# Round 3 GPU pass c: LDS kernel torus wrap + T = 48 ranks tests, then the
# LDS kernel and default benches.  Each step has its own limit.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03c
mkdir -p $O
step() {
  local name=$1 limit=$2
  shift 2
  timeout -k 10 "$limit" "$@"
  local rc=$?
  echo "step $name rc=$rc" >&2
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop" >&2; exit $rc; fi
  return 0
}
step tests 400 python -u -m pytest tests/test_gpu.py -q -k "lds or t48 or affinity or chain" --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
tail -3 $O/pytest.log
: > $O/bench.jsonl
step lds8192 200 env GOL_U8_KERNEL=lds python bench.py --layout u8 --size 8192 --steps 20 --warmup 2 --prewarm 2000 --verify 100 --no-phase-step >> $O/bench.jsonl 2>> $O/bench.err
step lds32768 200 env GOL_U8_KERNEL=lds python bench.py --layout u8 --size 32768 --steps 3 --warmup 1 --prewarm 200 --gens-per-step 100 --verify 0 --no-phase-step >> $O/bench.jsonl 2>> $O/bench.err
step default 300 python bench.py >> $O/bench.jsonl 2>> $O/bench.err
step tile 200 python bench.py --height 4096 --verify 0 --no-phase-step >> $O/bench.jsonl 2>> $O/bench.err
step tile_rccl 200 python bench.py --height 4096 --rehearse-rccl --verify 0 --no-phase-step >> $O/bench.jsonl 2>> $O/bench.err
python3 - <<'PY'
import json
for l in open("gpurun_out/r03c/bench.jsonl"):
    d = json.loads(l); c = d["config"]
    print("%-16s %-6s T=%-2d ep=%-4d %8.3f ms/step %.4g verified=%s %s" % (c["grid"], c["layout"], c["tmax"], c["epoch"], d["ms_per_step"], d["value"], d["verified"], c["overlap_mode"]))
PY
