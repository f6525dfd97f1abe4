set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_auto_blocks.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "auto_blocks or hybrid or gs" > gpurun_out/r03e_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03e_tests.log; [ $rc -eq 0 ] || exit $rc
for b in 4096 2048 1024; do
  HVE_AUTO_BLOCK_ROWS=$b timeout -k 10 300 python bench.py --n 256 --relax -1 --steps 10 --warmup 2 --cpu-cycles 0 --secondary-n 0 > gpurun_out/gs256_b$b.log 2>&1 || exit 1
  echo "level-0 blocks of $b rows: $(grep -h 'ms/step' gpurun_out/gs256_b$b.log)"
done
HVE_LAYOUT_LOG=1 timeout -k 10 600 python scripts/knob_ab.py 512 A1,A2,R1,R0 "" > gpurun_out/layout512.log 2>&1 || exit 1
grep -h "dict\|coded\|knobs" gpurun_out/layout512.log
