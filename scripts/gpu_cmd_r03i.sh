set -u
mkdir -p gpurun_out
for t in 1 0; do
  HVE_CODED_TILES=$t timeout -k 10 600 python scripts/knob_ab.py 512 R0,A1,R1 "" > gpurun_out/ctiles$t.log 2>&1 || exit 1
  echo "coded tiles $t: $(grep -h knobs gpurun_out/ctiles$t.log)"
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -q --timeout 600 --timeout-method thread -k "bench_size_256" > gpurun_out/r03i_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03i_tests.log; [ $rc -eq 0 ] || exit $rc
