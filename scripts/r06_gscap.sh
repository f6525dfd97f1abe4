# Pipelined GS sweep with a per-schedule unit capacity: the GS parity tests,
# then the launch variants of the hybrid-GS cycle at 256^3 and 512^3
# (scripts/gs_ab.py), with a kernel trace of the 256^3 A/B.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06/${1:-15_gschunk}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests -k "gs or hybrid or smoother or relax or pins or multirank" > $OUT/tests.txt 2>&1 && \
timeout -k 10 300 python -u scripts/gs_ab.py 256 > $OUT/ab256.txt 2>&1 && \
timeout -k 10 600 python -u scripts/gs_ab.py 512 > $OUT/ab512.txt 2>&1
echo "exit $?"
