#!/bin/bash
# Fused residual + restriction: parity tests, then the default bench (512^3,
# all parity legs) and a kernel trace of the 512^3 cycle.
set -u
OUT=gpurun_out/${TAG:-fused}
mkdir -p $OUT
export TMPDIR=/tmp
HVE_LAYOUT_LOG=${LLOG:-} timeout -k 10 400 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "fused_resid_restrict or single_cycle or sell_policy" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 900 python -u bench.py > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
grep "steps in\|parity\|setup parity\|fine SpMV" $OUT/bench.log
if [[ ${TRACE:-1} == 1 ]]; then
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python bench.py --secondary-n 0 --cpu-cycles 0 --steps 10 --warmup 2 --spmv-reps 5 > $OUT/trace.log 2>&1 \
  || { tail -20 $OUT/trace.log; exit 1; }
f=$(find $OUT/trace -name run_kernel_trace.csv | sort | tail -1)
python scripts/trace_summary.py $f 5 > $OUT/trace_summary.txt 2>&1
head -25 $OUT/trace_summary.txt
fi
