#!/bin/bash
# Round-3 final tier on the committed tree: smoke, full GPU tier, the driver's
# bench, the 8-GPU rank tile, u8 default, and kernel traces of the defaults.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/r03f
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "gpu tier rc=$rc"; grep -E "^FAILED|passed|failed" $O/pytest_gpu.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-240 $O/bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --height 4096 --steps 20 --warmup 5 > $O/bench_tile4096.json 2>> $O/bench.err
rc=$?; echo "tile rc=$rc"; cut -c1-200 $O/bench_tile4096.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --layout u8 --steps 10 --warmup 3 > $O/bench_u8.json 2>> $O/bench.err
rc=$?; echo "u8 rc=$rc"; cut -c1-200 $O/bench_u8.json; [ $rc -eq 0 ] || exit $rc
B="--steps 5 --warmup 1 --verify 0 --no-phase-step"
for spec in "bits:" "tile:--height 4096" "u8:--layout u8"; do
  name=${spec%%:*}; args=${spec#*:}
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$name -o run -- python3 bench.py $B $args > $O/trace_$name.json 2> $O/trace_$name.err
  rc=$?; echo "trace $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for name in bits tile u8; do echo "== $name"; f=$(find $O/trace_$name -name "*kernel_stats.csv" | head -1); head -5 "$f" | cut -c1-220; done
