set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_scale.py -k "out14 or out15 or out16" > gpurun_out/r03q_interp.log 2>&1 || { tail -40 gpurun_out/r03q_interp.log; exit 1; }
grep -E "grid|iterations|passed|failed" gpurun_out/r03q_interp.log
