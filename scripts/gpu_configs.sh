#!/bin/bash
# BASELINE configs[2] (BoomerAMG-PCG 512^3) and configs[4]'s method on one GPU
# (anisotropic 512^3, PMIS + 1 aggressive level) with the current layouts.
set -u
OUT=gpurun_out/configs
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-400
  case $rc in 0|1|2|5) return 0 ;; *) echo "=== stopping after $name (rc=$rc)"; exit $rc ;; esac
}
step pcg512 500 python bench.py --solver pcg --n 512 --secondary-n 0 --steps 10 --warmup 2 --cpu-cycles 0
step aniso_agg512 500 python bench.py --coef 0.001,1,1 --agg 1 --n 512 --secondary-n 0 --steps 10 --warmup 2
echo "=== done"
