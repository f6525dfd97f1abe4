#!/bin/bash
# BoomerAMG's default smoothers (hybrid GS 13/14, automatic blocks) and HMIS
# at 256^3 beside the bench line's l1-Jacobi / PMIS.
set -u
OUT=gpurun_out/smoothers
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$OUT/$name.log"
  case $rc in 0|1|2|5) return 0 ;; *) echo "=== stopping after $name (rc=$rc)"; exit $rc ;; esac
}
step hybrid_gs_256 400 python bench.py --n 256 --secondary-n 0 --relax -1 --steps 10 --warmup 2
step hmis_256 400 python bench.py --n 256 --secondary-n 0 --coarsen 10 --steps 10 --warmup 2
step stencil27_256 400 python bench.py --n 256 --secondary-n 0 --stencil 27 --steps 10 --warmup 2
echo "=== done"
