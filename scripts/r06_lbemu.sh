# The loopback N-rank bench lines at 128^3 (scripts/gpu_round.sh loop) against
# the one-GPU rank emulation of the same N ranks: bench.py --emulate 2 / 8.
set -o pipefail
OUT=gpurun_out/r06/${1:-32_lbemu}
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --emulate 2 --n 128 > $OUT/emulate2.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --emulate 8 --n 128 > $OUT/emulate8.txt 2>&1
echo "exit $?"
