#!/bin/bash
# Adder-window (GOL_XLANE=3) correctness tier and A/B bench against the DPP
# kernel on the full grid and on the 8-GPU per-rank tile.  Each GPU step has
# its own limit; the script stops at the first failure.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "adder or kernel_variants or u8_kernel_variants" > gpurun_out/pytest_adder.log 2>&1
tail -2 gpurun_out/pytest_adder.log
for x in 0 3 0 3; do
  GOL_XLANE=$x timeout -k 10 120 python bench.py --gpus 1 --steps 10 --warmup 2 >> gpurun_out/ab_full.jsonl 2>>gpurun_out/ab.err
  GOL_XLANE=$x timeout -k 10 120 python bench.py --gpus 1 --steps 10 --warmup 2 --height 4096 --epoch 256 >> gpurun_out/ab_tile.jsonl 2>>gpurun_out/ab.err
done
python3 - <<'PY'
import json
for f in ("gpurun_out/ab_full.jsonl", "gpurun_out/ab_tile.jsonl"):
    for l in open(f):
        d = json.loads(l)
        print(f.split("/")[-1], d["config"]["engine"].split("[")[1][:28], "%.3f ms/step" % d["ms_per_step"], "%.3g" % d["value"])
PY
