#!/bin/bash
# Occupancy and LDS evidence: one PMC pass per run of
# SQ_WAVES / SQ_WAVE_CYCLES / SQ_INSTS_VALU / GRBM_GUI_ACTIVE (calibrated on
# ubench_clock's exact 1 / 2 / 4 waves per SIMD), for the headline adder
# kernel, the 8-GPU rank tile, the byte layout's default deep pass and the
# LDS-tiled single-step byte kernel (plus its LDS counters), and a kernel
# trace of the byte layout at its current default.  Every step has its own
# limit; a step that does not end with 0 ends the script.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/occ
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
[ -x bin/ubench_clock ] || hipcc --offload-arch=gfx950 -O3 csrc/tools/ubench_clock.hip -o bin/ubench_clock
run clock 90 rocprofv3 --pmc $OCC --output-format csv -d $O/clock -o run -- bin/ubench_clock
run full 150 rocprofv3 --pmc $OCC --output-format csv -d $O/full -o run -- python3 bench.py $B
run tile 150 rocprofv3 --pmc $OCC --output-format csv -d $O/tile -o run -- python3 bench.py $B --height 4096
run u8 200 rocprofv3 --pmc $OCC --output-format csv -d $O/u8 -o run -- python3 bench.py $B --layout u8
export GOL_U8_KERNEL=lds
run lds 150 rocprofv3 --pmc $OCC --output-format csv -d $O/lds -o run -- python3 bench.py $B --layout u8 --size 8192 --gens-per-step 200 --prewarm 200
run lds_banks 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d $O/lds_banks -o run -- python3 bench.py $B --layout u8 --size 8192 --gens-per-step 200 --prewarm 200
unset GOL_U8_KERNEL
run u8_trace 200 rocprofv3 --kernel-trace --stats -d $O/u8_trace -o run -- python3 bench.py --layout u8 --steps 5 --warmup 1 --verify 0 --no-phase-step
echo all ok
