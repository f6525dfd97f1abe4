set -u
mkdir -p gpurun_out
for t in 1 0; do
  HVE_DICT_TILES_A2=$t timeout -k 10 600 python scripts/knob_ab.py 512 A2,J2,A1 "" > gpurun_out/a2t$t.log 2>&1 || exit 1
  echo "A2 tiles $t: $(grep -h knobs gpurun_out/a2t$t.log)"
done
