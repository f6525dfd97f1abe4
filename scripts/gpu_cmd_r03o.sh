set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "policy" > gpurun_out/r03o_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03o_tests.log; [ $rc -eq 0 ] || exit $rc
HVE_LAYOUT_LOG=1 HVE_SELL_CODED=0 HVE_SELL_DICT=1 timeout -k 10 600 python scripts/knob_ab.py 512 R0,R1,A1 "" > gpurun_out/r0dict.log 2>&1 || exit 1
echo "R0 dict+vt16: $(grep -h 'rows=41117982 group=1' gpurun_out/r0dict.log | head -1) $(grep -h knobs gpurun_out/r0dict.log)"
cat gpurun_out/rbands.log 2>/dev/null
