#!/bin/bash
# Grid-stencil loop on the ranks' interior rows: loopback parity tests, then
# the 8-rank loopback bench (256^3 global).
set -u
OUT=gpurun_out/${TAG:-gridm}
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?;
  grep -E "steps in|A0 residual|passed|failed|Error" $OUT/$name.log | head -20; echo "=== $name rc=$rc"; [[ $rc == 0 ]] || { tail -30 $OUT/$name.log; exit $rc; }; }
step tests 900 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "grid_stencil or stencil_layout or partitioned_27pt or out5"
step loopback8 600 python -u bench.py --loopback 8 --n 256 --secondary-n 0 --cpu-cycles 0 --steps 10 --warmup 2 --spmv-reps 5 --setup-parity 0 --pcg-iters 0
