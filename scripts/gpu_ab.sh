#!/bin/bash
# A/B of kernel variants on the full 32768^2 grid and the 8-GPU rank tile:
#   scripts/gpu_ab.sh "<label>:<env assignments>:<bench args>" ...
# Each configuration runs twice, interleaved; one JSON line per run in
# gpurun_out/ab.jsonl (label added).  Every GPU step has its own limit.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/ab.jsonl
for rep in 1 2; do
  for spec in "$@"; do
    IFS=: read -r label envs args <<< "$spec"
    out=$(env $envs timeout -k 10 150 python bench.py --gpus 1 --steps 10 --warmup 2 $args 2>>gpurun_out/ab.err)
    echo "{\"label\": \"$label\", \"rep\": $rep, \"run\": $out}" >> gpurun_out/ab.jsonl
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/ab.jsonl"):
    d = json.loads(l)
    r = d["run"]
    print("%-28s rep%d %8.3f ms/step %.3g" % (d["label"], d["rep"], r["ms_per_step"], r["value"]))
PY
