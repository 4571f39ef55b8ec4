#!/bin/bash
# PMC passes of the wide (1M x 64K) and tall (64K x 1M) 2^36-cell grids (round 6): why 128 KiB
# rows run 20 % slower per cell.  One counter set per run (TLB, L2, issue).
#   bash scripts/gpu_shape_pmc.sh OUTDIR
set -uo pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=${1:-gpurun_out/shape_pmc}
mkdir -p "$O"
B="--steps 1 --warmup 1 --prewarm 100 --verify 0 --no-phase-step"
run() {  # NAME COUNTERS bench-args...
  local name=$1 ctr=$2
  shift 2
  timeout -s KILL 180 rocprofv3 --pmc $ctr --output-format csv -d "$O/$name" -o run -- python3 bench.py "$@" \
    > "$O/$name.out" 2> "$O/$name.err"
  local rc=$?
  echo "pmc $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
TLB="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_PENDING_STALL_CYCLES_sum"
L2="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum"
ISS="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
for spec in "wide|--size 1048576 --height 65536" "tall|--size 65536 --height 1048576"; do
  n=${spec%%|*}; a=${spec#*|}
  run tlb_$n "$TLB" $B $a
  run l2_$n "$L2" $B $a
  run iss_$n "$ISS" $B $a
done
echo shape pmc done
