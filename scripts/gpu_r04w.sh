#!/bin/bash
# Round 4 batch w: config-2 bench (8192^2 byte layout, 20 steps, verified),
# the 8192^2 bits bench, and kernel traces without the oracle (--verify 0).
set -o pipefail
O=gpurun_out/r04w
mkdir -p "$O"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python bench.py --size 8192 --layout u8 --steps 20 --warmup 5 > $O/bench_8192_u8.json 2> $O/bench.err || exit $?
timeout -k 10 300 python bench.py --size 8192 --steps 20 --warmup 5 > $O/bench_8192_bits.json 2>> $O/bench.err || exit $?
timeout -k 10 300 python bench.py --height 4096 --rehearse-rccl --steps 20 --warmup 5 > $O/bench_tile_rehearsal.json 2>> $O/bench.err || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="--steps 5 --warmup 1 --verify 0 --no-phase-step"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/u8_8192 -o run -- python3 bench.py $B --size 8192 --layout u8 > $O/u8_8192.json 2> $O/u8_8192.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tile -o run -- python3 bench.py $B --height 4096 --rehearse-rccl > $O/tile.json 2> $O/tile.err
