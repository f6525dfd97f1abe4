# Coded-loop occupancy sweep (knob 2) for R_0 and P_0 at 512^3.
set -o pipefail
OUT=gpurun_out/r06/${1:-33_wpc}
mkdir -p $OUT
timeout -k 10 300 python -u scripts/code_wpc.py 512 > $OUT/wpc512.txt 2>&1
echo "exit $?"
