#!/bin/bash
# BASELINE config "8192^2 on 1 MI355X, LDS-tiled u8 kernel": kernel trace,
# LDS bank-conflict / occupancy counters and HBM bytes (separate passes;
# counters never combined with tracing).
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_lds
ARGS="--layout u8 --size 8192 --steps 300 --warmup 20"
export GOL_U8_KERNEL=lds
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lds/trace -o run -- python3 bench.py $ARGS > gpurun_out/prof_lds/bench_trace.json 2> gpurun_out/prof_lds/trace.err
timeout -k 10 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES --output-format csv -d gpurun_out/prof_lds/pmc_lds -o run -- python3 bench.py $ARGS > gpurun_out/prof_lds/pmc_lds.json 2> gpurun_out/prof_lds/pmc_lds.err
timeout -k 10 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_lds/pmc_fetch -o run -- python3 bench.py $ARGS > gpurun_out/prof_lds/pmc_fetch.json 2> gpurun_out/prof_lds/pmc_fetch.err
timeout -k 10 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_lds/pmc_write -o run -- python3 bench.py $ARGS > gpurun_out/prof_lds/pmc_write.json 2> gpurun_out/prof_lds/pmc_write.err
timeout -k 10 150 rocprofv3 --pmc SQ_LEVEL_WAVES SQ_ACCUM_PREV_HIRES --output-format csv -d gpurun_out/prof_lds/pmc_occ -o run -- python3 bench.py $ARGS > gpurun_out/prof_lds/pmc_occ.json 2> gpurun_out/prof_lds/pmc_occ.err
echo "lds profile done"
