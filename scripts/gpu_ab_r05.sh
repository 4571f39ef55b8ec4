# A/B of this tree against a round-5 checkout staged in r05_tree/ (not
# tracked): final-grid digests (scripts/digest_check.py) and bench.py on the
# headline, 8192^2 and the rehearsed 8-GPU rank tile, alternating trees.
O=gpurun_out/r06/ab2; mkdir -p $O
run() {  # run TREE NAME ARGS...
  local t=$1 n=$2; shift 2
  (cd $t && timeout -k 10 200 python bench.py --steps 10 --warmup 2 "$@") > $O/$n.json 2> $O/$n.err || { echo "FAIL $n"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', round(d['ms_per_step'],3), d['verified'])"
}
timeout -k 10 300 python -u scripts/digest_check.py > $O/digest_r06.txt 2>&1 && cat $O/digest_r06.txt || exit 1
for rep in 1 2; do
  for spec in "full|" "s8192|--size 8192" "tile8|--height 4096 --rehearse-rccl"; do
    n=${spec%%|*}; a=${spec#*|}
    run r05_tree r05_${n}_$rep $a
    run . r06_${n}_$rep $a
  done
done
