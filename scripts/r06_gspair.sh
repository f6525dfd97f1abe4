# Paired GS entry loads: the whole GPU suite, then the launch-variant A/B (paired / unpaired loads and the rest)
# of the hybrid-GS cycle at 256^3 and 512^3 (scripts/gs_ab.py).
set -o pipefail
OUT=gpurun_out/r06/${1:-13_gspair}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $OUT/tests.txt 2>&1 && \
timeout -k 10 300 python -u scripts/gs_ab.py 256 > $OUT/ab256.txt 2>&1 && \
timeout -k 10 500 python -u scripts/gs_ab.py 512 > $OUT/ab512.txt 2>&1
echo "exit $?"
