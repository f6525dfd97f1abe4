set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -q --timeout 600 --timeout-method thread -k "bench_size_256" > gpurun_out/r03l_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03l_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_l.log 2>&1 || exit 1
grep -h "ms/step\|A1 \|R1 \|parity" gpurun_out/bench_l.log
