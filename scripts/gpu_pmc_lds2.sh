#!/bin/bash
# Occupancy and LDS counters of the packed LDS tile at 8192^2: 16-wave
# workgroups (the default on this one-round grid) vs 8 (GOL_LDS_WAVES=8).
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/occ_lds2
mkdir -p $O
OCC="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
LDSC="SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
B="--steps 3 --warmup 1 --prewarm 200 --verify 0 --no-phase-step --layout u8 --u8-compute bytes --size 8192 --gens-per-step 256"
run() {  # run NAME LIMIT CMD...
  local name=$1 limit=$2
  shift 2
  timeout -s KILL "$limit" "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "step $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
[ -x bin/ubench_clock ] || hipcc --offload-arch=gfx950 -O3 csrc/tools/ubench_clock.hip -o bin/ubench_clock
run clock 90 rocprofv3 --pmc $OCC --output-format csv -d $O/clock -o run -- bin/ubench_clock
export GOL_U8_KERNEL=lds
run w16 150 rocprofv3 --pmc $OCC --output-format csv -d $O/w16 -o run -- python3 bench.py $B
run w16_lds 150 rocprofv3 --pmc $LDSC --output-format csv -d $O/w16_lds -o run -- python3 bench.py $B
export GOL_LDS_WAVES=8
run w8 150 rocprofv3 --pmc $OCC --output-format csv -d $O/w8 -o run -- python3 bench.py $B
run w8_lds 150 rocprofv3 --pmc $LDSC --output-format csv -d $O/w8_lds -o run -- python3 bench.py $B
echo all ok
