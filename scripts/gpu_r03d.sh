#!/bin/bash
# Chain hand-off fix check (forced chains), then the full GPU tier + smoke + bench.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03d
mkdir -p $O
GOL_U8_VIA_BITS=0 GOL_CHAIN=1 timeout -k 10 240 python -u scripts/chain_probe.py > $O/chain_probe.log 2>&1
rc=$?; echo "chain probe rc=$rc"; cut -c1-160 $O/chain_probe.log | tail -17
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "gpu tier rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest_gpu.log | tail -30; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 $O/bench.json
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_u8bits.sh
