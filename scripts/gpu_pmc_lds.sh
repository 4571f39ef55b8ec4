#!/bin/bash
# Occupancy and LDS counters of the LDS-tiled byte kernels at 8192^2 (BASELINE
# config 2): the packed tile (default, T = 32) and the byte tile (T = 8), one
# PMC pass per run, each step under its own limit.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/occ_lds
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
run packed 150 rocprofv3 --pmc $OCC --output-format csv -d $O/packed -o run -- python3 bench.py $B
run packed_lds 150 rocprofv3 --pmc $LDSC --output-format csv -d $O/packed_lds -o run -- python3 bench.py $B
export GOL_LDS_PACK=0
run bytes 150 rocprofv3 --pmc $OCC --output-format csv -d $O/bytes -o run -- python3 bench.py $B
run bytes_lds 150 rocprofv3 --pmc $LDSC --output-format csv -d $O/bytes_lds -o run -- python3 bench.py $B
unset GOL_LDS_PACK GOL_U8_KERNEL
run trace 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py $B
echo all ok
