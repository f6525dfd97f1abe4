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
  echo "=== $name rc=$rc"; tail -2 "$OUT/$name.log"
  case $rc in 0|1|2|5) return 0 ;; *) echo "=== stopping after $name (rc=$rc)"; exit $rc ;; esac
}
HVE_EXPER=4 step gatheronly 300 python scripts/ops_time.py 256
HVE_SELL_DICT_GROUP=8 step group8 300 python scripts/ops_time.py 256
echo "=== done"
