#!/bin/bash
# Grid-stencil workgroups of 16 waves (64x64 tiles) against 8: parity, 512^3.
set -u
OUT=gpurun_out/${TAG:-w16}
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?;
  grep -E "steps in|A0 residual|passed|failed|Error" $OUT/$name.log | head -6; echo "=== $name rc=$rc"; [[ $rc == 0 ]] || { tail -30 $OUT/$name.log; exit $rc; }; }
step tests16 600 env HVE_GRID_WAVES=16 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 200 --timeout-method thread -k grid_stencil
Q="--secondary-n 0 --cpu-cycles 0 --steps 20 --warmup 3 --spmv-reps 20 --setup-parity 0 --pcg-iters 0"
step b512_w16 600 env HVE_GRID_WAVES=16 python -u bench.py --n 512 $Q
step b512_w8 600 python -u bench.py --n 512 $Q
