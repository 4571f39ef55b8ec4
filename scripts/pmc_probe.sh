#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 5 120 rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
ARGS="--steps 300 --warmup 20"
for set in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES" "SQ_INST_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU_INT32 SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_MISC SQ_BUSY_CU_CYCLES"; do
  n=$(echo $set | cut -d' ' -f1)
  timeout -k 10 200 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc/$n -o run -- python3 bench.py $ARGS > gpurun_out/pmc/$n.json 2> gpurun_out/pmc/$n.err || echo "pmc set $n failed"
done
ls -R gpurun_out/pmc | head -40
