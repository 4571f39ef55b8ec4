#!/bin/bash
# Round 4 batch r: kernel traces of the linked 8192^2 defaults (bits and the
# byte layout), for profiles/r04/rocprof_kernel_traces_linked.md.
set -o pipefail
O=gpurun_out/r04r
mkdir -p "$O"
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="--steps 5 --warmup 1 --no-phase-step"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/bits8192 -o run -- python3 bench.py $B --size 8192 > $O/bits8192.json 2> $O/bits8192.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/u8_8192 -o run -- python3 bench.py $B --size 8192 --layout u8 > $O/u8_8192.json 2> $O/u8_8192.err
