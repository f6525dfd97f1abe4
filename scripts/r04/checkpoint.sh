#!/bin/bash
# Round-4 checkpoint on one box: the default bench line (parity legs and CPU
# baseline included), then the rocprofv3 trace and PMC traffic passes.
set -u
OUT=gpurun_out/${TAG:-ckpt}
mkdir -p $OUT
export TMPDIR=/tmp
echo "=== bench ($(date +%T))"
timeout -k 10 900 python -u bench.py > $OUT/bench.log 2>&1; rc=$?
echo "=== bench rc=$rc"; tail -c 1500 $OUT/bench.log
[[ $rc == 0 ]] || exit $rc
bash scripts/gpu_prof.sh all
