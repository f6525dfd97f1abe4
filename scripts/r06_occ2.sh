# Occupancy: the dictionary loop with fewer workgroups a CU (knob 17) at
# 512^3 (scripts/dict_occ.py), then the GS sweeps' default 8 KiB LDS pad
# against none and 16 KiB (scripts/gs_ab.py occ), after the GS tests.
set -o pipefail
OUT=gpurun_out/r06/${1:-23_occ2}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests -k "gs or hybrid or smoother or relax" > $OUT/tests.txt 2>&1 && \
timeout -k 10 400 python -u scripts/dict_occ.py 512 > $OUT/dict512.txt 2>&1 && \
timeout -k 10 300 python -u scripts/gs_ab.py 256 occ > $OUT/gs256.txt 2>&1 && \
timeout -k 10 500 python -u scripts/gs_ab.py 512 occ > $OUT/gs512.txt 2>&1
echo "exit $?"
