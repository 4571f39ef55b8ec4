#!/bin/bash
# Parameter sweep of the 1-GPU bench; one JSON line per configuration.
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/sweep.jsonl
: > $OUT
run() {
  echo "== $*" >&2
  if ! timeout -k 10 240 env "$@" >> $OUT 2>> gpurun_out/sweep.err; then echo "FAILED: $*" >&2; exit 1; fi
}
for cfg in "${SWEEP[@]}"; do
  eval "run $cfg"
done
cat $OUT
