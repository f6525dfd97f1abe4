#!/bin/bash
# Default 8-wave grid-stencil workgroups: parity tests, then the rocprofv3
# trace and PMC traffic passes over the default bench (scripts/gpu_prof.sh).
set -u
OUT=gpurun_out/${TAG:-w8}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_scale.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -k "grid_stencil or bench_size or 27pt or aniso or fused_resid or pcg" > $OUT/tests.log 2>&1 \
  || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash scripts/gpu_prof.sh all
