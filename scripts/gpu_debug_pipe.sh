#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/dbg
timeout -k 10 300 python -u scripts/debug_pipe_u8.py > gpurun_out/dbg/pipe48.txt 2>&1; echo rc=$?
cat gpurun_out/dbg/pipe48.txt | tail -40
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -q -k "t48 or deep_byte" --timeout 300 --timeout-method thread > gpurun_out/dbg/pytest_t48.log 2>&1; echo rc=$?
tail -5 gpurun_out/dbg/pytest_t48.log
