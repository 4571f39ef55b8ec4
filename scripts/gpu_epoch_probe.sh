cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06/ktrace
mkdir -p $O
for n in plain trigger; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/$n -o run -- python3 bench.py --height 4096 --rehearse-rccl --overlap $( [ $n = plain ] && echo off || echo trigger ) --steps 5 --warmup 1 --no-phase-step --verify 0 > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  f=$(find $O/$n -name "*kernel_trace.csv" | head -1)
  echo "== $n"; python3 scripts/epoch_gaps.py $f; python3 scripts/launch_gaps.py $f | head -6
done
