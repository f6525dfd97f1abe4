set -u
mkdir -p gpurun_out
true
true
HVE_SETUP_T=1 timeout -k 10 900 python scripts/setup_phases.py 512 > gpurun_out/setup512.log 2>&1 || exit 1
grep -v "^level" gpurun_out/setup512.log | tail -20
