#!/bin/bash
set -u
mkdir -p gpurun_out/exp
OUT=gpurun_out/exp
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$OUT/$name.log"
  case $rc in 0|1|2|5) return 0 ;; *) echo "=== stopping after $name (rc=$rc)"; exit $rc ;; esac
}
step dictp_tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread -k "policy or bench_size or 27pt or aniso"
step pipe256 300 python scripts/ops_time.py 256
HVE_DICT_PIPE=0 step nopipe256 300 python scripts/ops_time.py 256
step pipe512 400 python scripts/ops_time.py 512
echo "=== done"
