#!/bin/bash
# quick check: solve-loop parity tests + 512^3 op/iteration timing
set -u
OUT=gpurun_out/quick
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "$OUT/$name.log"
  case $rc in 0|1|2|5) return 0 ;; *) echo "=== stopping after $name (rc=$rc)"; exit $rc ;; esac
}
step tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 300 --timeout-method thread
step ops512 500 python scripts/ops_time.py ${N:-512}
echo "=== done"
