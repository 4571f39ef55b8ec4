#!/bin/bash
# Multi-rank checks on the one-GPU box: the shared-GPU RCCL tests (2, 4 and 8
# real rank processes on CU partitions), the linking rule of the multi-rank
# schedule, and bench.py --gpus 8 --share-gpus at the headline grid.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=gpurun_out/${1:-r05/multirank}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_rccl_multirank.py tests/test_gpu.py -x -v --timeout 600 \
  --timeout-method thread -k "rccl or multirank or links_only or rehearsal or share" > $O/pytest.log 2>&1 \
  || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 600 python -u bench.py --gpus 8 --share-gpus --steps 3 --warmup 1 --prewarm 2000 --verify 96 \
  > $O/bench_8ranks_shared.json 2> $O/bench_8ranks_shared.err || { tail -40 $O/bench_8ranks_shared.err; exit 1; }
cat $O/bench_8ranks_shared.json
