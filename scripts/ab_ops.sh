#!/bin/bash
# A/B of level-operator timings (scripts/ops_time.py) between in-tree library
# builds, plus the GPU parity tests on the default build.  One gpurun call:
#   bash scripts/ab_ops.sh N lib_dirA lib_dirB ...   (TESTS=0 skips the tests)
set -u
OUT=gpurun_out/ab
mkdir -p $OUT
export TMPDIR=/tmp
N=$1; shift
step() {
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$OUT/$name.log"
  case $rc in 0|1|2|5) return 0 ;; *) echo "=== stopping after $name (rc=$rc)"; exit $rc ;; esac
}
if [[ ${TESTS:-1} == 1 ]]; then
  step tests 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread
fi
for L in "$@"; do
  HVE_LIB_PATH=hypre-ve_amd/$L/libhypreve.so step ops_${N}_$L 600 python scripts/ops_time.py $N
done
echo "=== done"
