#!/bin/bash
# Dictionary loop with buffer loads and two register sets: parity tests, then
# 512^3 per-kernel timings (A1, R1, A2).
set -u
OUT=gpurun_out/${TAG:-dict}
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?;
  grep -E "steps in|A0 residual|A1 resid|R1 restr|A2 resid|R0 restr|P0 prol|P1 prol|passed|failed|Error" $OUT/$name.log | head -20; echo "=== $name rc=$rc"; [[ $rc == 0 ]] || { tail -30 $OUT/$name.log; exit $rc; }; }
step tests 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "sell_policy or single_cycle or pcg or grid_stencil or interp_types or aggressive or hybrid_gs_cycle or loopback_partitioned or coded or fused_resid"
Q="--secondary-n 0 --cpu-cycles 0 --steps 20 --warmup 3 --spmv-reps 20 --setup-parity 0 --pcg-iters 0"
step b512 600 python -u bench.py --n 512 $Q
step gs512 900 python -u bench.py --n 512 --relax -1 $Q
