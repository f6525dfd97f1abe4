# The RAP fill in two launches too (small and full tables): the whole GPU
# suite (device setup == host setup), the 512^3 setup phases (HVE_SETUP_T),
# then the bench line.
set -o pipefail
OUT=gpurun_out/r06/${1:-30_rap2}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/tests.txt 2>&1 && \
HVE_SETUP_T=1 timeout -k 10 400 python -u scripts/setup_phases.py 512 > $OUT/setup512.txt 2>&1 && \
timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 > $OUT/bench.txt 2>&1
echo "exit $?"
