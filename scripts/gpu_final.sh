#!/bin/bash
# Smoke, the driver's default bench (twice), the per-rank tiles of the 2/4/8-GPU
# split (local fill and RCCL rehearsal), and a kernel-trace profile of the
# default bench.  Every GPU step has its own limit.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
echo smoke ok
: > gpurun_out/final.jsonl
for i in 1 2; do
  timeout -k 10 200 python bench.py >> gpurun_out/final.jsonl 2>>gpurun_out/final.err
done
for args in "--height 16384" "--height 8192" "--height 4096" \
            "--height 16384 --rehearse-rccl" "--height 8192 --rehearse-rccl" "--height 4096 --rehearse-rccl"; do
  timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 $args >> gpurun_out/final.jsonl 2>>gpurun_out/final.err
done
python3 - <<'PY'
import json
for l in open("gpurun_out/final.jsonl"):
    d = json.loads(l); c = d["config"]
    print("%-12s %-32s %-28s T=%-2d ep=%-4d steps=%-3d %8.3f ms/step %.4g" % (c["grid"], c["kernel"], c["parallelism"][:28], c["tmax"], c["epoch"], d["steps"], d["ms_per_step"], d["value"]))
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run -- python3 bench.py --steps 5 --warmup 1 > gpurun_out/prof_final.json 2> gpurun_out/prof_final.err
cat gpurun_out/prof_final.json
