#!/bin/bash
# Attribution of the 8-GPU rank tile's in-kernel gap:
# PMC passes (one counter set per run; rocprofv3 serialises the launches, so
# linked launches run alone here) of the ring tile 32768 x 4096 (DPP T = 16,
# waves of 2T rows: all prologue / epilogue triangle, no steady loop), of the
# same DPP T = 16 kernel on the full grid (long waves: the steady-state rate
# at the same code) and of config 2's 8192^2; per-wave traces of a linked
# launch pair on the tile; and the tile's T sweep in the timed bench.
#   bash scripts/gpu_attrib.sh OUTDIR
set -uo pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=${1:-gpurun_out/attrib}
mkdir -p "$O"
pmc() {  # NAME COUNTERS bench.py-args...
  local name=$1 ctr=$2
  shift 2
  timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d "$O/$name" -o run -- python3 bench.py "$@" \
    > "$O/$name.out" 2> "$O/$name.err"
  local rc=$?
  echo "pmc $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
OCC="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
ISS="SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
B="--steps 2 --warmup 1 --prewarm 1024 --verify 0 --no-phase-step"
for spec in "tile8ring|--height 4096" "fulldpp16|--tune xlane=0 --tmax 16" "s8192|--size 8192"; do
  n=${spec%%|*}; a=${spec#*|}
  pmc occ_$n "$OCC" $B $a
  pmc iss_$n "$ISS" $B $a
done
python3 scripts/occupancy.py "tile8_ring=$O/occ_tile8ring" "full_32768_dpp_T16=$O/occ_fulldpp16" "s8192_bits=$O/occ_s8192" \
  > "$O/occupancy.md" 2> "$O/occupancy.err" || echo "occupancy.py failed"
python3 scripts/attrib.py "$O" > "$O/attrib.md" 2> "$O/attrib.err" || echo "attrib.py failed"
# Per-wave records of launches 300 and 301 (linked) on the ring tile.
GOL_WG_TRACE="100:$O/wg_tile8_pair.csv:pair" timeout -k 10 120 python3 bench.py --height 4096 $B > "$O/wg.out" 2> "$O/wg.err" || { tail -5 "$O/wg.err"; exit 1; }
python3 scripts/wg_trace.py --pair "$O/wg_tile8_pair.csv" > "$O/wg_tile8_pair.txt" 2>&1 || echo "wg_trace.py failed"
# T sweep of the tile (DPP window), timed.
timeout -k 10 400 python3 -u scripts/bench_matrix.py scripts/matrices/main.txt "$O/tsweep.jsonl" --timeout 120 \
  --only tile8_ring,tile8_ring_T12,tile8_ring_T8,tile8_rehearsal,tile8_rehearsal_T12 || exit 1
echo attrib done
