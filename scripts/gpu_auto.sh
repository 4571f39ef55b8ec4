#!/bin/bash
# Full GPU tier, smoke, and the default (auto kernel policy) bench on the full
# grid and the per-rank tiles of the 2/4/8-GPU strong-scaling split.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
echo smoke ok
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
tail -2 gpurun_out/pytest_gpu.log
: > gpurun_out/auto.jsonl
for args in "" "--height 16384" "--height 8192" "--height 4096"; do
  timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 $args >> gpurun_out/auto.jsonl 2>>gpurun_out/auto.err
done
python3 - <<'PY'
import json
for l in open("gpurun_out/auto.jsonl"):
    d = json.loads(l); c = d["config"]
    print("%-12s %-30s T=%-2d ep=%-4d %8.3f ms/step %.3g" % (c["grid"], c["kernel"], c["tmax"], c["epoch"], d["ms_per_step"], d["value"]))
PY
