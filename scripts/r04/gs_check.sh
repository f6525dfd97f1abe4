#!/bin/bash
# Hybrid Gauss-Seidel on the packed schedule: the GS parity tests, then the
# relax 13/14 V-cycle at N^3 under a kernel trace for each team size.
set -u
OUT=gpurun_out/${TAG:-gs_check}
mkdir -p $OUT
export TMPDIR=/tmp
if [[ ${TESTS:-1} == 1 ]]; then
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_reference_pins.py tests/test_gpu_multirank.py \
  -k "hybrid or default_smoothers or rank_fixture or fixture_default or cf_relax" > $OUT/tests.log 2>&1 \
  || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
fi
N=${N:-256}
for T in ${TEAMS:-64}; do
  HVE_GS_TEAM_ROWS=$T timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/trace_t$T -o run --output-format csv -- \
    python bench.py --n $N --secondary-n 0 --cpu-cycles 0 --relax -1 --steps 10 --warmup 2 --spmv-reps 5 \
    > $OUT/bench_t$T.log 2>&1 || { tail -20 $OUT/bench_t$T.log; exit 1; }
  f=$(find $OUT/trace_t$T -name run_kernel_trace.csv | sort | tail -1)
  python scripts/trace_summary.py $f 5 > $OUT/trace_summary_t$T.txt 2>&1
  echo "== team_rows $T"; grep "steps in" $OUT/bench_t$T.log; grep "k_hybrid" $OUT/trace_summary_t$T.txt | head -12
done
