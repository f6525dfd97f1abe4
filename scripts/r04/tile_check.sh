#!/bin/bash
# Tiled level-0 restriction (k_tile_restrict): parity tests, then 512^3 with
# and without it on the same box.
set -u
OUT=gpurun_out/${TAG:-tile}
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?;
  grep -E "steps in|A0 residual|R0 restr|passed|failed" $OUT/$name.log; echo "=== $name rc=$rc"; [[ $rc == 0 ]] || { tail -30 $OUT/$name.log; exit $rc; }; }
step tests 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "${TESTK:-fused_resid or grid_stencil or sell_policy or single_cycle or pcg or large_solve}"
Q="--secondary-n 0 --cpu-cycles 0 --steps 20 --warmup 3 --spmv-reps 20 --setup-parity 0 --pcg-iters 0"
step b512_tile 600 python -u bench.py --n 512 $Q
step b512_notile 600 env HVE_TILE_R=0 python -u bench.py --n 512 $Q
