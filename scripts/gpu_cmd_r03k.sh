set -u
mkdir -p gpurun_out
: > gpurun_out/tileshape2.log
for sh in "128,4,2:" "256,2,2:" "256,4,1:" "512,2,1:" "128,4,2:64,8,8" "128,4,2:128,8,4" "128,4,2:256,4,4"; do
  t1=${sh%%:*}; t2=${sh##*:}
  HVE_DICT_TILE=$t1 HVE_DICT_TILE2=$t2 timeout -k 10 600 python scripts/knob_ab.py 512 A1,J1,R1 "" > gpurun_out/ts.log 2>&1 || exit 1
  echo "tile '$sh': $(grep -h knobs gpurun_out/ts.log)" | tee -a gpurun_out/tileshape2.log
done
