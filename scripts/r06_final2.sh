# The round's profiles at 512^3: a kernel trace of the bench's headline line
# alone (no secondary sizes, so each kernel's average is the 512^3 launch's),
# PMC traffic of the cycle's kernels (scripts/pmc_cycle.sh, the bench's
# roofline.traffic), then the per-operator table of A1, R1, A2, R0
# (scripts/gpu_opprof.sh).  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof512
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof512 -o run --output-format csv -- \
  python3 bench.py --steps 10 --warmup 2 --cpu-cycles 0 --secondary-n 0 --gs-n 0 > gpurun_out/prof512/bench.log 2>&1 && \
N=512 bash scripts/pmc_cycle.sh && \
OUT=gpurun_out/opprof512 N=512 OPS=A1,R1,A2,R0 bash scripts/gpu_opprof.sh
echo "exit $?"
