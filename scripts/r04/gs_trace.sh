#!/bin/bash
# Kernel trace of the hybrid Gauss-Seidel V-cycle (relax 13/14, automatic
# blocks) at N^3: where a GS cycle's time goes, per kernel and grid.
set -u
N=${N:-256}
OUT=gpurun_out/${TAG:-gs_trace}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python bench.py --n $N --secondary-n 0 --cpu-cycles 0 --relax -1 --steps 5 --warmup 1 --spmv-reps 5 \
  > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
f=$(find $OUT/trace -name run_kernel_trace.csv | sort | tail -1)
python scripts/trace_summary.py $f 5 > $OUT/trace_summary.txt 2>&1
tail -3 $OUT/bench.log; head -40 $OUT/trace_summary.txt
