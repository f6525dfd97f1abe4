# R_0's jagged, product-parallel coded loop (k_code_pw): the layout parity
# tests (policy 15 forces it), then an A/B at 512^3 against the padded loop
# (HVE_CODE_PW 0 / 1, scripts/ops_time.py, one process each).
set -o pipefail
OUT=gpurun_out/r06/${1:-09_r0pw}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "sell_policy" > $OUT/tests.txt 2>&1 && \
HVE_CODE_PW=0 timeout -k 10 200 python -u scripts/ops_time.py 512 > $OUT/pw0.txt 2>&1 && \
HVE_CODE_PW=1 timeout -k 10 200 python -u scripts/ops_time.py 512 > $OUT/pw1.txt 2>&1
echo "exit $?"
