#!/bin/bash
# Kernel-trace + stats profile of the 1-GPU bench, then a separate PMC pass.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
ARGS=${BENCH_ARGS:-"--steps 20 --warmup 2"}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- python3 bench.py $ARGS > gpurun_out/prof/bench_trace.json 2> gpurun_out/prof/bench_trace.err
echo "trace ok"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/prof/pmc1 -o run -- python3 bench.py $ARGS > gpurun_out/prof/bench_pmc1.json 2> gpurun_out/prof/bench_pmc1.err
echo "pmc1 ok"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY --output-format csv -d gpurun_out/prof/pmc2 -o run -- python3 bench.py $ARGS > gpurun_out/prof/bench_pmc2.json 2> gpurun_out/prof/bench_pmc2.err
echo "pmc2 ok"
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d gpurun_out/prof/pmc3 -o run -- python3 bench.py $ARGS > gpurun_out/prof/bench_pmc3.json 2> gpurun_out/prof/bench_pmc3.err || echo "pmc3 (icache) unavailable"
find gpurun_out/prof -name "*.csv" | head -50
