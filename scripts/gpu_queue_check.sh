#!/bin/bash
# Kernel traces of N separate bench processes on 8192^2 (round 6): which hardware queues the
# linked streams got, against each run's time (scripts/queue_check.py).
#   bash scripts/gpu_queue_check.sh OUTDIR [N] [bench args...]
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=${1:-gpurun_out/qcheck}; N=${2:-6}; shift 2
mkdir -p "$O"
for i in $(seq 1 "$N"); do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$O/r$i" -o run -- python3 bench.py "$@" \
    > "$O/r$i.json" 2> "$O/r$i.err" || { echo "run $i failed"; exit 1; }
done
python3 scripts/queue_check.py "$O"/r[0-9] "$O"/r[0-9][0-9] 2>/dev/null
