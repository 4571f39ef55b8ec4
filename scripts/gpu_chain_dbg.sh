#!/bin/bash
# Re-run the GPU tests that timed out in a chained-group wait (r03 full tier).
set -uo pipefail
export TMPDIR=/tmp GOL_U8_VIA_BITS=0
O=gpurun_out/chaindbg
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread \
  -k "every_temporal_block_size or adder_window or chained_groups" > $O/a.log 2>&1
rc=$?; echo "default rc=$rc"; tail -3 $O/a.log
[ $rc -le 1 ] || exit $rc
GOL_CHAIN=0 timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -q --timeout 120 --timeout-method thread \
  -k "every_temporal_block_size or adder_window" > $O/b.log 2>&1
rc=$?; echo "chain off rc=$rc"; tail -3 $O/b.log
