set -o pipefail
O=gpurun_out/r06/chain; mkdir -p $O
export GOL_TUNE_LOG=1
for spec in "full|" "fullu8|--layout u8" "s8192|--size 8192" "tile8|--height 4096 --rehearse-rccl" "tile4|--height 8192 --rehearse-rccl" "tile2|--height 16384 --rehearse-rccl" "s65536|--size 65536 --steps 1 --warmup 1"; do
  n=${spec%%|*}; a=${spec#*|}
  timeout -k 10 150 python3 bench.py --steps 3 --warmup 2 $a > $O/$n.json 2> $O/$n.err || { echo "step $n failed"; exit 1; }
  echo "$n: $(grep -c chained $O/$n.err) autotune lines, picks: $(grep -o -- '-> [a-z]*' $O/$n.err | sort | uniq -c | tr '\n' ' ')"
done
