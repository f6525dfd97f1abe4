set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_setup.py -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r03f_tests.log 2>&1; rc=$?; tail -15 gpurun_out/r03f_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/setup_phases.py 256 > gpurun_out/setup256.log 2>&1 || exit 1
grep -v "^level" gpurun_out/setup256.log | tail -6
