set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "interp_types" > gpurun_out/r03s_parity.log 2>&1 || { tail -40 gpurun_out/r03s_parity.log; exit 1; }
tail -2 gpurun_out/r03s_parity.log
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_scale.py -k "out17 or out18" > gpurun_out/r03s_bands.log 2>&1 || { tail -40 gpurun_out/r03s_bands.log; exit 1; }
grep -E "grid|iterations|passed|failed" gpurun_out/r03s_bands.log
