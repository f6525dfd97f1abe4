#!/bin/bash
# The default bench line with the final round-4 library.
set -u
OUT=gpurun_out/${TAG:-final}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py > $OUT/bench.log 2>&1; rc=$?
echo "=== bench rc=$rc"; grep -E "steps in|A0 residual|R0|P0|A1" $OUT/bench.log | head; exit $rc
