#!/bin/bash
# Per-wave placement/timing of one grouped launch (GOL_WG_TRACE) on the
# 8-GPU per-rank tile, the 4-GPU tile and the full grid.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/wgtrace
for cfg in "4096" "8192" "32768"; do
  GOL_WG_TRACE=10:$R/gpurun_out/wgtrace/h$cfg.csv timeout -k 10 120 python3 $R/bench.py --size 32768 --height $cfg \
    --steps 200 --warmup 20 > $R/gpurun_out/wgtrace/h$cfg.json
  for t in ${WG_TARGETS:-}; do
    GOL_TARGET_WAVES=$t GOL_WG_TRACE=10:$R/gpurun_out/wgtrace/h${cfg}_t$t.csv timeout -k 10 120 python3 $R/bench.py \
      --size 32768 --height $cfg --steps 200 --warmup 20 > $R/gpurun_out/wgtrace/h${cfg}_t$t.json
  done
done
python3 $R/scripts/wg_trace.py $R/gpurun_out/wgtrace/*.csv
