# A 10-step GS ring (HVE_GS_RING=10: 5 KiB a wave instead of 8, four
# workgroups a CU) against the default 16, the hybrid-GS cycle at 256^3 and
# 512^3 (scripts/gs_ab.py, default launch; the iterate sha must agree).
set -o pipefail
OUT=gpurun_out/r06/${1:-21_ring10}
mkdir -p $OUT
L10=hypre-ve_amd/lib_r10/libhypreve.so
timeout -k 10 300 python -u scripts/gs_ab.py 256 quick > $OUT/ab256.txt 2>&1 && \
HVE_LIB_PATH=$L10 timeout -k 10 300 python -u scripts/gs_ab.py 256 quick > $OUT/ab256_r10.txt 2>&1 && \
timeout -k 10 400 python -u scripts/gs_ab.py 512 quick > $OUT/ab512.txt 2>&1 && \
HVE_LIB_PATH=$L10 timeout -k 10 400 python -u scripts/gs_ab.py 512 quick > $OUT/ab512_r10.txt 2>&1
echo "exit $?"
