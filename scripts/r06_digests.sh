set -o pipefail
mkdir -p gpurun_out/r06/01_digests
timeout -k 10 900 python -u bench.py --coef 0.001,1,1 --agg 1 --steps 10 --warmup 2 --secondary-n 0 --setup-parity 0 --pcg-iters 0 > gpurun_out/r06/01_digests/agg512.log 2>&1 && \
timeout -k 10 200 python -u bench.py --stencil 27 --steps 2 --warmup 1 --secondary-n 0 --setup-parity 0 --pcg-iters 0 > gpurun_out/r06/01_digests/b27_512.log 2>&1
echo "exit $?"
