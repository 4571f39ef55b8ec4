#!/bin/bash
# PMC passes (one counter set per run) of the flow and grouped launches on
# 32768^2: occupancy / VALU issue, SALU and wait counters, instruction cache.
set -uo pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=gpurun_out/${1:-r05/pmc_flow}
mkdir -p $O
B="--steps 2 --warmup 1 --prewarm 1024 --verify 0 --no-phase-step"
run() {  # run NAME CMD...
  local name=$1
  shift
  timeout -s KILL 120 "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "step $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
OCC="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
ISS="SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
for f in 0 1; do
  export GOL_FLOW=$f
  run occ_full_f$f rocprofv3 --pmc $OCC --output-format csv -d $O/occ_full_f$f -o run -- python3 bench.py $B
  run iss_full_f$f rocprofv3 --pmc $ISS --output-format csv -d $O/iss_full_f$f -o run -- python3 bench.py $B
done
for f in 1 0; do
  export GOL_FLOW=$f
  run icache_full_f$f rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS --output-format csv -d $O/icache_full_f$f -o run -- python3 bench.py $B
done
echo all ok
