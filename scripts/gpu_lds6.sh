#!/bin/bash
# Packed LDS tile at its 160-row default: exactness (LDS tests) and config 2.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/lds6
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -k "lds" -q --timeout 120 --timeout-method thread > $O/pytest_lds.log 2>&1
rc=$?; echo "lds tests rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest_lds.log | tail -8; [ $rc -eq 0 ] || exit $rc
GOL_U8_KERNEL=lds timeout -k 10 200 python bench.py --layout u8 --u8-compute bytes --size 8192 --steps 20 --warmup 2 > $O/bench_8192_lds.json 2>> $O/err.log
rc=$?; echo "8192 lds rc=$rc"; cut -c1-400 $O/bench_8192_lds.json; [ $rc -eq 0 ] || exit $rc
