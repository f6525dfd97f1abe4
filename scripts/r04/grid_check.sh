#!/bin/bash
# Grid-stencil loop (k_grid_stencil): parity tests, then the finest passes at
# 512^3 (7-point) and one rank's 27-point 8-GPU share, with and without it.
set -u
OUT=gpurun_out/${TAG:-grid}
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?;
  tail -c 300 $OUT/$name.log; echo; echo "=== $name rc=$rc"; [[ $rc == 0 ]] || exit $rc; }
step tests 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "${TESTK:-grid_stencil or pcg_ij_64 or fused_resid or wide_stride}"
Q="--secondary-n 0 --cpu-cycles 0 --steps 20 --warmup 3 --spmv-reps 20 --setup-parity 0 --pcg-iters 0"
step b512_grid 600 python -u bench.py --n 512 $Q
step b512_slice 600 env HVE_GRID_STENCIL=0 python -u bench.py --n 512 $Q
step s27_grid 600 env OMP_NUM_THREADS=16 python -u bench.py --grid 512,512,64 --stencil 27 $Q
step s27_slice 600 env OMP_NUM_THREADS=16 HVE_GRID_STENCIL=0 python -u bench.py --grid 512,512,64 --stencil 27 $Q
