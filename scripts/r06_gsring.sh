# 16-lane GS ring slots for the wide operators' schedules: the GS parity tests
# (run while 16 was the default), then the hybrid-GS cycle with 64- and 16-lane
# rings (knob 14 at setup) at 256^3 and 512^3 (scripts/gs_ab.py, default
# launch; iterate sha printed).
set -o pipefail
OUT=gpurun_out/r06/${1:-17_gsring}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests -k "gs or hybrid or smoother or relax or pins or multirank" > $OUT/tests.txt 2>&1 && \
timeout -k 10 300 python -u scripts/gs_ab.py 256 rw16 quick > $OUT/ab256.txt 2>&1 && \
timeout -k 10 300 python -u scripts/gs_ab.py 256 quick > $OUT/ab256_rw64.txt 2>&1 && \
timeout -k 10 400 python -u scripts/gs_ab.py 512 rw16 quick > $OUT/ab512.txt 2>&1 && \
timeout -k 10 400 python -u scripts/gs_ab.py 512 quick > $OUT/ab512_rw64.txt 2>&1
echo "exit $?"
