# R_0's jagged coded loop with the next chunk's codes prefetched: parity of
# the launch variants (knobs 4 / 5), then the padded loop's R_0 and the
# jagged variants at 512^3 (scripts/r0_pw_knobs.py, one process each).
set -o pipefail
OUT=gpurun_out/r06/${1:-11_r0wpc}
mkdir -p $OUT
true && \
timeout -k 10 200 python -u scripts/r0_pw_knobs.py 512 > $OUT/pw0.txt 2>&1 && \
timeout -k 10 200 python -u scripts/r0_pw_knobs.py 512 jag > $OUT/pw1.txt 2>&1
echo "exit $?"
