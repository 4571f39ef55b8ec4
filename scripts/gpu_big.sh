#!/bin/bash
# GPU tier + default bench + roctx marker trace + large-grid memory check.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/big
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
cat gpurun_out/bench.json
python -c "import torch; p=torch.cuda.get_device_properties(0); f,t=torch.cuda.mem_get_info(); print('device mem total', p.total_memory, 'free', f, t)"
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d gpurun_out/big/marker -o run -- python3 bench.py --steps 256 --warmup 64 > gpurun_out/big/marker_bench.json 2> gpurun_out/big/marker.err
echo "marker trace ok"
timeout -k 10 600 python bench.py --layout u8 --size 1048576 --height 65536 --steps 8 --warmup 2 > gpurun_out/big/u8_1M_x65536.json 2> gpurun_out/big/u8_1M.err
cat gpurun_out/big/u8_1M_x65536.json
