#!/bin/bash
# Chained-group give-up probe: default spin bound, then 64x longer.
set -uo pipefail
export TMPDIR=/tmp GOL_U8_VIA_BITS=0 GOL_CHAIN=1
O=gpurun_out/chainprobe
mkdir -p $O
timeout -k 10 240 python -u scripts/chain_probe.py > $O/spin16.log 2>&1
rc=$?; echo "spin16 rc=$rc"; cat $O/spin16.log | cut -c1-220
[ $rc -le 1 ] || exit $rc
GOL_CHAIN_SPIN=22 timeout -k 10 240 python -u scripts/chain_probe.py > $O/spin22.log 2>&1
rc=$?; echo "spin22 rc=$rc"; cat $O/spin22.log | cut -c1-220
