# Counter passes of the round: PMC traffic of the cycle's kernels at 512^3
# (scripts/pmc_cycle.sh, the bench's roofline.traffic), then the per-operator
# table of A1, R1, A2, R0 (scripts/gpu_opprof.sh).  Stops at the first failure.
set -o pipefail
N=512 bash scripts/pmc_cycle.sh && \
OUT=gpurun_out/opprof512 N=512 OPS=A1,R1,A2,R0 bash scripts/gpu_opprof.sh
echo "exit $?"
