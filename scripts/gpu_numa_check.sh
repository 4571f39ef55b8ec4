#!/bin/bash
# 8192^2 spread against the host NUMA node the process runs on (round 6):
# three bench processes pinned (taskset) to the CPUs of each NUMA node this
# process may use, plus three unpinned ones, each recording its median.
#   bash scripts/gpu_numa_check.sh [OUT]
set -o pipefail
out=${1:-gpurun_out/r06/numa}
mkdir -p "$out"
{ lscpu | grep -i -E 'numa|socket|model name'; timeout -k 10 60 python3 scripts/numa_cpus.py; } > "$out/topo.txt" 2>&1 || exit $?
cat "$out/topo.txt"
args="--size 8192 --layout u8 --steps 50 --warmup 10 --no-phase-step"
while read -r tag node cpus; do
  [ "$tag" = node ] || continue
  # a few CPUs of the node are enough for one bench process
  pick=$(echo "$cpus" | cut -d, -f1-8)
  for i in 1 2 3; do
    timeout -k 10 120 taskset -c "$pick" python3 bench.py $args > "$out/node${node}_$i.json" 2> "$out/node${node}_$i.err" || exit $?
    echo "node $node run $i: $(python3 -c 'import json,sys; print(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["ms_per_step"])' "$out/node${node}_$i.json")"
  done
done < "$out/topo.txt"
for i in 1 2 3; do
  timeout -k 10 120 python3 bench.py $args > "$out/free_$i.json" 2> "$out/free_$i.err" || exit $?
  echo "unpinned run $i: $(python3 -c 'import json,sys; print(json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["ms_per_step"])' "$out/free_$i.json")"
done
