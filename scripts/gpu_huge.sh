#!/bin/bash
# BASELINE config 5 capacity checks on one GPU (288 GiB HBM3E):
#  * the per-GPU share of the 8-GPU 1,048,576^2 byte-per-cell run (1048576 x 131072 u8,
#    double-buffered = 2 x 137.6 GB), and
#  * the WHOLE 1,048,576^2 grid in the bit layout (2 x 137.4 GB).
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/huge
timeout -k 10 900 python bench.py --layout u8 --size 1048576 --height 131072 --steps 16 --warmup 2 > gpurun_out/huge/u8_1M_x131072.json 2> gpurun_out/huge/u8.err
cat gpurun_out/huge/u8_1M_x131072.json
timeout -k 10 900 python bench.py --layout bits --size 1048576 --steps 32 --warmup 16 > gpurun_out/huge/bits_1M_square.json 2> gpurun_out/huge/bits.err
cat gpurun_out/huge/bits_1M_square.json
