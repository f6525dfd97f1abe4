set -u
mkdir -p gpurun_out
true
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 1 --dist --grid 128,128,128 --steps 50 --warmup 3 --cpu-cycles 0 > gpurun_out/dist128.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --n 128 --steps 50 --warmup 3 --cpu-cycles 0 --secondary-n 0 > gpurun_out/plain128.log 2>&1 || exit 1
grep -h "ms/step" gpurun_out/dist128.log gpurun_out/plain128.log
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --cpu-cycles 0 --secondary-n 0 > gpurun_out/bench512.log 2>&1 || exit 1
grep -h "\[bench\]" gpurun_out/bench512.log | tail -12
VARIANTS="HVE_STENCIL_WMAP=0 HVE_STENCIL_WMAP=1 HVE_STENCIL_R=2" bash scripts/gpu_stencil_ab.sh
