#!/bin/bash
# One rank's share of configs[4] (anisotropic + aggressive, 512x512x64) with
# the final kernels and the 2 host threads an 8-rank node leaves a rank.
set -u
OUT=gpurun_out/${TAG:-shareagg}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 env OMP_NUM_THREADS=2 python -u bench.py --grid 512,512,64 --coef 0.001,1,1 --agg 1 --secondary-n 0 \
  --cpu-cycles 0 --steps 20 --warmup 3 --spmv-reps 10 --setup-parity 0 --pcg-iters 0 > $OUT/shareagg.log 2>&1; rc=$?
grep -E "steps in|A0 residual" $OUT/shareagg.log; exit $rc
