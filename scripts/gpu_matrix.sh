#!/bin/bash
# Parametrised GPU batch: optional pytest selection, then one bench matrix.
#   bash scripts/gpu_matrix.sh MATRIX OUT.jsonl [PYTEST_ARGS...]
# PYTEST_ARGS empty: no tests.  Every step has its own time limit; a failing
# step ends the batch (no further GPU work).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
m=$1; out=$2; shift 2
mkdir -p "$(dirname "$out")"
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread "$@" \
    > "${out%.jsonl}_pytest.log" 2>&1 || { tail -60 "${out%.jsonl}_pytest.log"; exit 1; }
  tail -3 "${out%.jsonl}_pytest.log"
fi
timeout -k 10 1000 python -u scripts/bench_matrix.py "$m" "$out" --timeout 150
