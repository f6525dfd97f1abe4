# Kernel breakdown of the hybrid-GS cycle (relax 13 / 14, BoomerAMG's
# default smoothers) at 256^3: rocprofv3 kernel trace of 10 solve iterations.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06/${1:-12_gs256}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o gs -- \
  python3 -u scripts/cycle_trace.py 256 10 relax_type=-1 > $OUT/run.txt 2>&1 && \
python3 scripts/trace_summary.py $(find $OUT/trace -name '*kernel_trace.csv' | sort | tail -n 1) 10 > $OUT/summary.txt
echo "exit $?"
