# Round-6 checkpoint on one MI355X, each step under its own time limit,
# stopping at the first failure: the layout parity tests, the multi-rank
# tests (N-rank contract, reference np > 1 runs through the distributed
# setup), the default 512^3 bench line.
set -o pipefail
OUT=gpurun_out/r06/${1:-03_contract}
mkdir -p $OUT
T="python -u -m pytest -x -v --timeout 250 --timeout-method thread -m gpu"
timeout -k 10 400 $T tests/test_gpu_parity.py -k "sell_policy or matvec" > $OUT/tests_parity.txt 2>&1 && \
timeout -k 10 700 $T tests/test_gpu_multirank.py tests/test_gpu_multiprocess.py > $OUT/tests_multirank.txt 2>&1 && \
timeout -k 10 500 python -u bench.py --steps 20 --warmup 3 --secondary-n 0 --setup-parity 0 > $OUT/bench512.txt 2>&1
echo "exit $?"
