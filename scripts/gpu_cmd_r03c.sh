set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 300 --timeout-method thread -k "policy or coded" > gpurun_out/r03c_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03c_tests.log; [ $rc -eq 0 ] || exit $rc
S=";0=2;0=2,1=4;0=4;1=4;1=16;2=4;2=16;0=2,2=4;0=2,2=16"
timeout -k 10 300 python scripts/knob_ab.py 256 P0,R0 "$S" > gpurun_out/knob256.log 2>&1 || exit 1
HVE_SELL_CODED=0 timeout -k 10 300 python scripts/knob_ab.py 256 P0,R0 "" > gpurun_out/knob256_old.log 2>&1 || exit 1
cat gpurun_out/knob256.log gpurun_out/knob256_old.log
