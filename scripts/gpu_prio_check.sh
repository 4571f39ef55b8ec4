#!/bin/bash
# GPU tests + wave traces (priority on / off) + 1-GPU bench after the wave-priority change.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/wgtrace
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/pytest_gpu.log 2>&1
for h in 4096 32768; do
  GOL_WG_TRACE=10:$R/gpurun_out/wgtrace/on$h.csv timeout -k 10 60 python3 bench.py --size 32768 --height $h --steps 200 --warmup 20 > /dev/null
  GOL_NATIVE_SO=alt_so/prio0/_gol.so GOL_WG_TRACE=10:$R/gpurun_out/wgtrace/off$h.csv timeout -k 10 60 python3 bench.py --size 32768 --height $h --steps 200 --warmup 20 > /dev/null
done
timeout -k 10 120 python3 bench.py > $R/gpurun_out/bench_default.json
