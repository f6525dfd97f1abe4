set -u
mkdir -p gpurun_out
timeout -k 10 300 python scripts/stencil_ab.py --n 512 --settings "6=1;;5=4;5=12;5=16;6=1" --tag pp > gpurun_out/pp512.log 2>&1 || exit 1
cat gpurun_out/pp512.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread -k "policy or stencil or wide_stride or bench_size_256 or 27pt or pcg or cycle or matvec" > gpurun_out/r03d_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03d_tests.log; [ $rc -eq 0 ] || exit $rc
