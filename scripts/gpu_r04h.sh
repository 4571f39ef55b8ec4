#!/bin/bash
# Round 4 batch h: PMC occupancy / VALU issue passes (one counter set per run)
# for the round-4 defaults: 8192^2 byte layout (T = 8, 4-wave groups, row
# ring), the 8-GPU rank tile, the headline; LDS counters of the grouped
# kernel at 8192^2.  Summarised by scripts/occupancy.py.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04h}
mkdir -p $O
OCC="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
B="--steps 3 --warmup 1 --prewarm 2048 --verify 0 --no-phase-step"
run() {  # run NAME LIMIT CMD...
  local name=$1 limit=$2
  shift 2
  timeout -s KILL "$limit" "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "step $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
run u8_8192 150 rocprofv3 --pmc $OCC --output-format csv -d $O/u8_8192 -o run -- python3 bench.py $B --size 8192 --layout u8
run tile 150 rocprofv3 --pmc $OCC --output-format csv -d $O/tile -o run -- python3 bench.py $B --height 4096
run full 150 rocprofv3 --pmc $OCC --output-format csv -d $O/full -o run -- python3 bench.py $B
run lds_8192 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d $O/lds_8192 -o run -- python3 bench.py $B --size 8192
echo all ok
