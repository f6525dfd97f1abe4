set -u
mkdir -p gpurun_out
for t in 1 0; do
  HVE_LAYOUT_LOG=1 HVE_DICT_TILES=$t timeout -k 10 600 python scripts/knob_ab.py 512 A1,A2,R1,P1 "" > gpurun_out/tiles$t.log 2>&1 || exit 1
  echo "tiles $t: $(grep -h 'group=' gpurun_out/tiles$t.log | head -3 | tr '\n' ' ') $(grep -h knobs gpurun_out/tiles$t.log)"
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -q --timeout 600 --timeout-method thread -k "bench_size_256" > gpurun_out/r03h_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03h_tests.log; [ $rc -eq 0 ] || exit $rc
