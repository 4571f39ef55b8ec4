#!/bin/bash
# Per-run pack of the byte layout on bit words: GPU tier, u8 measurements, kernel traces.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03e
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "gpu tier rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest_gpu.log | tail -30; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_u8bits.sh || exit $?
bash scripts/gpu_trace_r03.sh
