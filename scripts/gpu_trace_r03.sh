#!/bin/bash
# Kernel traces (csv) of the headline bits run, the byte layout at its
# current default (epochs on bit words) and on the byte kernels (T = 48
# pipelined pairs), and the 8-GPU rank tile.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/trace
mkdir -p $O
B="--steps 5 --warmup 1 --verify 0 --no-phase-step"
for spec in "bits:" "u8:--layout u8" "u8bytes:--layout u8 --u8-compute bytes" "tile:--height 4096" \
            "tile_rccl:--height 4096 --rehearse-rccl"; do
  name=${spec%%:*}; args=${spec#*:}
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$name -o run -- python3 bench.py $B $args > $O/$name.json 2> $O/$name.err
  rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for name in bits u8 u8bytes tile tile_rccl; do echo "== $name"; head -6 $O/$name/run_kernel_stats.csv | cut -c1-200; done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err
rc=$?; echo "bench rc=$rc"; cut -c1-260 $O/bench_default.json
