#!/bin/bash
# Round 3 GPU pass: the multi-rank RCCL tests (ranks sharing one GPU),
# device-affinity checks, the full GPU tier, and the default bench with its
# verification gate and per-phase step.  Every GPU step has its own limit; a
# step that times out, aborts or faults ends the script (test failures do not).
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03a
step() {  # step NAME LIMIT CMD...: run, and stop the script unless rc is 0 or 1
  local name=$1 limit=$2
  shift 2
  timeout -k 10 "$limit" "$@"
  local rc=$?
  echo "step $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "step $name ended with rc=$rc: no further GPU steps"
    exit $rc
  fi
  return 0
}
step multirank 400 python -u -m pytest tests/test_rccl_multirank.py -v --timeout 300 --timeout-method thread \
  > gpurun_out/r03a/pytest_multirank.log 2>&1
tail -3 gpurun_out/r03a/pytest_multirank.log
step gpu_tier 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  --deselect tests/test_rccl_multirank.py > gpurun_out/r03a/pytest_gpu.log 2>&1
tail -3 gpurun_out/r03a/pytest_gpu.log
step bench 300 python bench.py > gpurun_out/r03a/bench.json 2> gpurun_out/r03a/bench.err
cat gpurun_out/r03a/bench.json
step bench_u8 300 python bench.py --layout u8 --steps 5 --warmup 1 > gpurun_out/r03a/bench_u8.json \
  2> gpurun_out/r03a/bench_u8.err
cat gpurun_out/r03a/bench_u8.json
