#!/bin/bash
# Round 4 batch n: the whole GPU tier with linked launches on by default, the
# driver's smoke, and the default bench plus BASELINE config 2.
set -o pipefail
OUT=gpurun_out/${1:-r04n}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 700 --timeout-method thread -m gpu tests \
  > "$OUT/tier.log" 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
timeout -k 10 300 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || exit $?
timeout -k 10 300 python bench.py --size 8192 --layout u8 --steps 20 --warmup 5 > "$OUT/bench_8192_u8.json" 2>> "$OUT/bench_default.err"
