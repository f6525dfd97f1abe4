# One-GPU references of the N-rank lines (bench.py --emulate N: the N-rank setup
# under the rank emulation, its iterate checked bit for bit against the C
# oracle, the slab digests that scripts/golden_digests.py merges), each under
# its own time limit, stopping at the first failure.
#   bash scripts/r06_refs.sh OUTDIR "bench args" N1 N2 ...
set -o pipefail
OUT=gpurun_out/r06/$1
ARGS=$2
shift 2
mkdir -p $OUT
rc=0
for N in "$@"; do
  timeout -k 10 ${REF_TIMEOUT:-380} python -u bench.py $ARGS --emulate $N > $OUT/emulate$N.txt 2>&1 || { rc=$?; break; }
done
echo "exit $rc"
