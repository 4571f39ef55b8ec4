set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out/probe
for n in 2 4; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2950$n scripts/rccl_shared_gpu_probe.py > gpurun_out/probe/n$n.out 2> gpurun_out/probe/n$n.err || { echo "n=$n failed rc=$?"; tail -30 gpurun_out/probe/n$n.err; exit 1; }
  cat gpurun_out/probe/n$n.out
done
