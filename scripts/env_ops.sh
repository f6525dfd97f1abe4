#!/bin/bash
# scripts/ops_time.py under several environment settings (one gpurun call):
#   bash scripts/env_ops.sh N "VAR=a,VAR2=b" "VAR=c" ...   ("base" = no change)
set -u
OUT=gpurun_out/envops
mkdir -p $OUT
export TMPDIR=/tmp
N=$1; shift
for v in "$@"; do
  e=""; [[ $v != base ]] && e=${v//,/ }
  name=${v//[=,]/_}
  echo "=== $v ($(date +%T))"
  timeout -k 10 400 env $e python scripts/ops_time.py $N > $OUT/$name.log 2>&1
  rc=$?
  echo "=== $v rc=$rc"; tail -1 $OUT/$name.log | cut -c1-600
  case $rc in 0) ;; *) echo "=== stopping (rc=$rc)"; exit $rc ;; esac
done
echo "=== done"
