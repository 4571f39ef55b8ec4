#!/bin/bash
# Round 4 batch z: the whole GPU tier on the committed tree (linked launches
# wherever two fit), the experimental module's tests, smoke(), and the
# driver's default bench command.
set -o pipefail
OUT=gpurun_out/${1:-r04z}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 700 --timeout-method thread -m gpu tests \
  > "$OUT/tier.log" 2>&1 || exit $?
GOL_NATIVE_SO=exp_so/_gol.so timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  -m "gpu and experimental" tests/test_gpu.py > "$OUT/experimental.log" 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
timeout -k 10 300 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err"
