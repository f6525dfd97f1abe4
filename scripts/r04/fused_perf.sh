#!/bin/bash
# Fused residual + restriction: its parity tests, then a kernel trace of the
# 512^3 bench cycle with it on (HVE_FUSE_RR=1) for the per-kernel times.
set -u
OUT=gpurun_out/${TAG:-fused_perf}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "fused_resid_restrict" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
HVE_FUSE_RR=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python bench.py --n ${N:-512} --secondary-n 0 --cpu-cycles 0 --steps 10 --warmup 2 --spmv-reps 5 > $OUT/trace.log 2>&1 \
  || { tail -20 $OUT/trace.log; exit 1; }
f=$(find $OUT/trace -name run_kernel_trace.csv | sort | tail -1)
python scripts/trace_summary.py $f 5 > $OUT/trace_summary.txt 2>&1
grep "steps in" $OUT/trace.log; grep "resid_restrict\|k_sell_stencil<0\|k_sell_code<6" $OUT/trace_summary.txt
