set -u
mkdir -p gpurun_out
: > gpurun_out/rbands.log
for b in 32 128 512 8; do
  HVE_BLOCK_ORDER_R=$b timeout -k 10 600 python scripts/knob_ab.py 512 R0,R1 "" > gpurun_out/rb.log 2>&1 || exit 1
  echo "R bands $b: $(grep -h knobs gpurun_out/rb.log)" | tee -a gpurun_out/rbands.log
done
