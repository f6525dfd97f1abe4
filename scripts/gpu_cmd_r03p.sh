set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "policy and (13 or 8 or 12)" > gpurun_out/r03p_tests.log 2>&1 || { tail -30 gpurun_out/r03p_tests.log; exit 1; }
tail -3 gpurun_out/r03p_tests.log
: > gpurun_out/pack.log
for cfg in "HVE_SELL_PACK=0" "HVE_SELL_PACK=1" "HVE_SELL_PACK=1 HVE_SELL_CODED=0"; do
  env $cfg timeout -k 10 600 python scripts/knob_ab.py 512 P0,R0,P1 "" > gpurun_out/pk.log 2>&1 || { tail gpurun_out/pk.log; exit 1; }
  echo "$cfg: $(grep -h knobs gpurun_out/pk.log)" | tee -a gpurun_out/pack.log
done
