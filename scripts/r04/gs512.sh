#!/bin/bash
# BoomerAMG's default smoothers (hybrid GS 13/14) at 512^3 on one GPU.
set -u
OUT=gpurun_out/${TAG:-gs512}
mkdir -p $OUT
export TMPDIR=/tmp
HVE_GS_TEAM_ROWS=${TEAM:-16} timeout -k 10 900 python -u bench.py --n 512 --secondary-n 0 --cpu-cycles 0 --relax -1 \
  --steps 5 --warmup 1 --spmv-reps 5 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep "steps in\|setup" $OUT/bench.log | head; tail -c 600 $OUT/bench.log
