set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_reference_pins.py -k "interp_types or rank_fixture" > gpurun_out/r03t.log 2>&1 || { tail -30 gpurun_out/r03t.log; exit 1; }
tail -3 gpurun_out/r03t.log
