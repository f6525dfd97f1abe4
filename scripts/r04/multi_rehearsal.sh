#!/bin/bash
# Multi-GPU rehearsals on one GPU: per-cycle halo exchanges on 8 loopback
# ranks (256^3 global), and one rank's share of the 8-GPU configs[3] / [4]
# runs (512 x 512 x 64) with the host threads an 8-rank node leaves a rank.
set -u
OUT=gpurun_out/${TAG:-multi}
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?;
  tail -c 400 $OUT/$name.log; echo; echo "=== $name rc=$rc"; [[ $rc == 0 ]] || exit $rc; }
step loopback8 600 python -u bench.py --loopback 8 --n 256 --secondary-n 0 --cpu-cycles 0 --steps 10 --warmup 2 --spmv-reps 5
step share27 900 env OMP_NUM_THREADS=${OMP_SHARE:-2} python -u bench.py --grid 512,512,64 --stencil 27 --secondary-n 0 --cpu-cycles 0 --steps 10 --warmup 2 --spmv-reps 5
step shareagg 900 env OMP_NUM_THREADS=${OMP_SHARE:-2} python -u bench.py --grid 512,512,64 --coef 0.001,1,1 --agg 1 --secondary-n 0 --cpu-cycles 0 --steps 10 --warmup 2 --spmv-reps 5
