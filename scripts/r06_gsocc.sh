# Fewer hybrid-GS workgroups a CU (knob 16: extra LDS a workgroup) at 256^3
# and 512^3 (scripts/gs_ab.py occ; every variant's iterate bitwise the default's).
set -o pipefail
OUT=gpurun_out/r06/${1:-22_gsocc}
mkdir -p $OUT
timeout -k 10 300 python -u scripts/gs_ab.py 256 occ > $OUT/ab256.txt 2>&1 && \
timeout -k 10 500 python -u scripts/gs_ab.py 512 occ > $OUT/ab512.txt 2>&1
echo "exit $?"
