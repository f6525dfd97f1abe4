#!/bin/bash
# Grid-stencil workgroups of 4 vs 8 waves (tiles 64x16 vs 64x32): parity with
# both, then 512^3 and the 27-point share with both.
set -u
OUT=gpurun_out/${TAG:-waves}
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?;
  grep -E "steps in|A0 residual|passed|failed|Error" $OUT/$name.log | head -8; echo "=== $name rc=$rc"; [[ $rc == 0 ]] || { tail -30 $OUT/$name.log; exit $rc; }; }
T="python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 200 --timeout-method thread -k grid_stencil"
step tests4 600 $T
step tests8 600 env HVE_GRID_WAVES=8 $T
Q="--secondary-n 0 --cpu-cycles 0 --steps 20 --warmup 3 --spmv-reps 20 --setup-parity 0 --pcg-iters 0"
step b512_w8 600 env HVE_GRID_WAVES=8 python -u bench.py --n 512 $Q
step b512_w4 600 python -u bench.py --n 512 $Q
step s27_w8 600 env HVE_GRID_WAVES=8 python -u bench.py --grid 512,512,64 --stencil 27 $Q
step s27_w4 600 python -u bench.py --grid 512,512,64 --stencil 27 $Q
