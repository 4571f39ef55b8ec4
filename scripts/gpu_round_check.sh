#!/bin/bash
# One GPU call for a round's evidence on the current tree: the whole GPU tier,
# the multi-rank rehearsals (scripts/gpu_multirank.sh), the 1M^2 verified run
# and the kernel-trace profiles (scripts/gpu_profile_round.sh).  Each step has
# its own time limit; the first failure ends the batch.
#   bash scripts/gpu_round_check.sh OUTDIR [steps]   (steps: any of tier,multirank,large,prof; default all)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=${1:-gpurun_out/check}
S=${2:-tier,multirank,large,prof}
mkdir -p "$O"
has() { [[ ",$S," == *",$1,"* ]]; }
if has tier; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
  tail -2 "$O/pytest_gpu.log"
fi
if has multirank; then
  bash scripts/gpu_multirank.sh "${O#gpurun_out/}/multirank" || exit 1
fi
if has large; then
  timeout -k 10 420 python -u scripts/bench_matrix.py scripts/matrices/main.txt "$O/large_1M.jsonl" --only bits_1M,u8_1M_share8 \
    --timeout 400 || exit 1
fi
if has prof; then
  bash scripts/gpu_profile_round.sh "$O/prof" || exit 1
fi
echo "round check done"
