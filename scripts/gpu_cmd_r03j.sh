set -u
mkdir -p gpurun_out
HVE_SETUP_T=1 timeout -k 10 900 python scripts/setup_phases.py 512 > gpurun_out/setup512w.log 2>&1 || exit 1
grep -h "dsetup\] extpi fill\|setup phases\|setup:\|setup total" gpurun_out/setup512w.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_setup.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r03j_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03j_tests.log; [ $rc -eq 0 ] || exit $rc
