#!/bin/bash
# Round 4 batch g: the experimental module's GPU tests, the default GPU tier,
# smoke(), and the driver's 1-GPU bench command.
set -o pipefail
OUT=gpurun_out/${1:-r04g}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
GOL_NATIVE_SO=exp_so/_gol.so timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  -m "gpu and experimental" tests/test_gpu.py > "$OUT/experimental_tier.log" 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > "$OUT/tier.log" 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_driver_args.json" 2> "$OUT/bench.err" || exit $?
