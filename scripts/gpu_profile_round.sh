#!/bin/bash
# Kernel traces (rocprofv3 --kernel-trace --stats) of the default build on the
# configurations the docs quote: the headline 32768^2, the 8-GPU rank tile in
# its multi-rank schedule (one-rank RCCL rehearsal) and BASELINE config 2
# (8192^2 byte layout); each summarised to markdown by summarize_profile.py.
#   bash scripts/gpu_profile_round.sh OUTDIR        (e.g. gpurun_out/r05/prof)
# Every run has its own time limit; a failing run ends the batch.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=${1:-gpurun_out/prof}
mkdir -p "$O"
run() {  # name, bench.py arguments...
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$n" -o run -- \
    python3 bench.py "$@" > "$O/$n.json" 2> "$O/$n.err" || { tail -30 "$O/$n.err"; return 1; }
  python3 scripts/summarize_profile.py "$O/$n" > "$O/$n.md" || return 1
  echo "$n ok: $(python3 -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(r['ms_per_step'], r['value'], r.get('verified'))" "$O/$n.json")"
}
run full_32768 --steps 10 --warmup 2 --no-phase-step &&
run tile_8gpu_rehearsal --height 4096 --rehearse-rccl --steps 10 --warmup 2 --no-phase-step &&
run config2_8192_u8 --size 8192 --layout u8 --steps 20 --warmup 5 --no-phase-step
