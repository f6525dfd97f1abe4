#!/bin/bash
# A/B of stencil-kernel variants (scripts/stencil_ab.py), one process each;
# every step under its own time limit, nothing further after a failure.
set -u
mkdir -p gpurun_out
OUT=gpurun_out/stencil_ab.log
: > $OUT
run() {
  echo "=== $*" >> $OUT
  timeout -k 10 300 env "$@" >> $OUT 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "=== rc=$rc, stopping" >> $OUT; tail -20 $OUT; exit $rc; fi
}
N=${N:-512}
for v in ${VARIANTS:-"HVE_STENCIL_WMAP=0" "HVE_STENCIL_WMAP=1"}; do
  run $v python scripts/stencil_ab.py --n $N --tag "$v"
done
cat $OUT
