#!/bin/bash
# 8 real RCCL ranks sharing one GPU (CU partitions) at the headline grid: the default poll
# placement (trial) against polls forced joined and forced side, alternating (round 6).
#   bash scripts/gpu_share8_poll_ab.sh OUTDIR
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
O=${1:-gpurun_out/share8_poll}
mkdir -p "$O"
for i in 1 2; do
  for m in auto 0 1; do
    if [ "$m" = auto ]; then unset GOL_SIDE_POLL; else export GOL_SIDE_POLL=$m; fi
    timeout -k 10 300 python -u bench.py --gpus 8 --share-gpus --steps 3 --warmup 1 --prewarm 2000 --verify 0 \
      --overlap off > "$O/poll_${m}_$i.json" 2> "$O/poll_${m}_$i.err" || { tail -20 "$O/poll_${m}_$i.err"; exit 1; }
    python3 -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=r['config']; print(sys.argv[2], r['ms_per_step'], c['poll_mode'], c['poll_trial_ms_per_window'], c.get('prewarm_trial_generations'))" "$O/poll_${m}_$i.json" "$m" || exit 1
  done
done
