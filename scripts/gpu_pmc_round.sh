#!/bin/bash
# PMC passes of the default build on the configurations the docs quote: the
# headline 32768^2, the 8-GPU rank tile in its multi-rank schedule (one-rank
# RCCL rehearsal) and BASELINE config 2 (8192^2 byte layout).  Two counter
# sets per configuration, one rocprofv3 run each (occupancy, issue); then
# scripts/occupancy.py writes the summary.
#   bash scripts/gpu_pmc_round.sh OUTDIR        (e.g. gpurun_out/r05/pmc)
set -uo pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=${1:-gpurun_out/pmc}
mkdir -p "$O"
run() {  # run NAME COUNTERS bench.py-args...
  local name=$1 ctr=$2
  shift 2
  timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d "$O/$name" -o run -- python3 bench.py "$@" \
    > "$O/$name.out" 2> "$O/$name.err"
  local rc=$?
  echo "step $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
OCC="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
ISS="SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
B="--steps 2 --warmup 1 --prewarm 1024 --verify 0 --no-phase-step"
for spec in "full|" "tile8|--height 4096 --rehearse-rccl" "config2|--size 8192 --layout u8"; do
  n=${spec%%|*}; a=${spec#*|}
  run occ_$n "$OCC" $B $a
  run iss_$n "$ISS" $B $a
done
python3 scripts/occupancy.py "full_32768=$O/occ_full" "tile8_rehearsal=$O/occ_tile8" "config2_8192_u8=$O/occ_config2" \
  > "$O/occupancy.md" 2> "$O/occupancy.err" || echo "occupancy.py failed (see .err)"
echo all ok
