# A/B of the lane-packed dictionary loop's variants at 512^3 (scripts/ops_time.py,
# one process per library build): the default, both register sets loaded
# before the x-tile gather (lib_A), 5 waves a SIMD (lib_B), both (lib_C).
set -o pipefail
OUT=gpurun_out/r06/${1:-07_ab_dictw}
mkdir -p $OUT
timeout -k 10 200 python -u scripts/ops_time.py 512 > $OUT/main.txt 2>&1 && \
HVE_LIB_PATH=hypre-ve_amd/lib_A/libhypreve.so timeout -k 10 200 python -u scripts/ops_time.py 512 > $OUT/pre2.txt 2>&1 && \
HVE_LIB_PATH=hypre-ve_amd/lib_B/libhypreve.so timeout -k 10 200 python -u scripts/ops_time.py 512 > $OUT/waves5.txt 2>&1 && \
HVE_LIB_PATH=hypre-ve_amd/lib_C/libhypreve.so timeout -k 10 200 python -u scripts/ops_time.py 512 > $OUT/pre2_waves5.txt 2>&1
echo "exit $?"
