#!/bin/bash
# Planes per grid-stencil workgroup (HVE_GRID_ZC) at 512^3: 16 / 64 against
# the default (32 with 8-wave tiles).
set -u
OUT=gpurun_out/${TAG:-zc}
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?;
  grep -E "steps in|A0 residual" $OUT/$name.log | head -4; echo "=== $name rc=$rc"; [[ $rc == 0 ]] || { tail -30 $OUT/$name.log; exit $rc; }; }
Q="--secondary-n 0 --cpu-cycles 0 --steps 20 --warmup 3 --spmv-reps 30 --setup-parity 0 --pcg-iters 0"
step zc_def 600 python -u bench.py --n 512 $Q
step zc16 600 env HVE_GRID_ZC=16 python -u bench.py --n 512 $Q
step zc64 600 env HVE_GRID_ZC=64 python -u bench.py --n 512 $Q
