# Strength and PMIS on the device: the device-setup tests (every level against
# the host setup, byte for byte), then the 512^3 setup split into its phases
# with the device stages timed (HVE_SETUP_T), then the bench line.
set -o pipefail
OUT=gpurun_out/r06/${1:-19_devpmis}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_setup.py > $OUT/tests.txt 2>&1 && \
HVE_SETUP_T=1 timeout -k 10 400 python -u scripts/setup_phases.py 512 > $OUT/setup512.txt 2>&1 && \
timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 > $OUT/bench.txt 2>&1
echo "exit $?"
