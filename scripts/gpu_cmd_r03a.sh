set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py tests/test_auto_blocks.py -m gpu -x -q --timeout 300 --timeout-method thread -k "rccl or partitioned_solve or auto_blocks" > gpurun_out/mr_tests.log 2>&1; rc=$?; tail -3 gpurun_out/mr_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 1 --dist --n 128 --steps 50 --warmup 3 --cpu-cycles 0 > gpurun_out/dist128.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --n 128 --steps 50 --warmup 3 --cpu-cycles 0 --secondary-n 0 > gpurun_out/plain128.log 2>&1 || exit 1
grep -h "ms/step" gpurun_out/dist128.log gpurun_out/plain128.log
VARIANTS="HVE_STENCIL_WMAP=0 HVE_STENCIL_WMAP=1 HVE_STENCIL_R=2" bash scripts/gpu_stencil_ab.sh
