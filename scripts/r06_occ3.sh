# The GS sweeps' LDS pad per level (run with a since-removed knob 18 that
# padded the level-0 sweep alone: none / 16 KiB for it gave the same times),
# after the GS tests; scripts/gs_ab.py occ now runs the uniform pad variants.
set -o pipefail
OUT=gpurun_out/r06/${1:-24_occ3}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests -k "gs or hybrid or smoother or relax" > $OUT/tests.txt 2>&1 && \
timeout -k 10 300 python -u scripts/gs_ab.py 256 occ > $OUT/gs256.txt 2>&1 && \
timeout -k 10 500 python -u scripts/gs_ab.py 512 occ > $OUT/gs512.txt 2>&1
echo "exit $?"
