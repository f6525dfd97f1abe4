#!/bin/bash
# Sourced by the GPU run scripts: `step NAME SECONDS CMD...` runs CMD under its
# own time limit with output in $OUT/NAME.log, and ends the script after a
# fault, abort, segfault or time limit (no further GPU step in that call).
set -u
OUT=${OUT:-gpurun_out/run}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -4 "$OUT/$name.log"
  case $rc in 0|1|2|5) return 0 ;; *) echo "=== stopping after $name (rc=$rc)"; exit $rc ;; esac
}
