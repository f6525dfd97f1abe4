#!/bin/bash
# A/B end-to-end bench on one box: bench.py under each env variant, alternated
# twice.  Usage: VARIANTS="X=0 Y=1,Z=2" bash scripts/ab_bench.sh [steps]
set -u
mkdir -p gpurun_out/ab
STEPS=${1:-20}
for round in 1 2; do
  for v in base ${VARIANTS}; do
    e=""; [[ $v != base ]] && e=${v//,/ }
    timeout -k 10 300 env $e python bench.py --steps $STEPS --warmup 3 --cpu-cycles 0 --spmv-reps 10 \
      > gpurun_out/ab/$v.$round.log 2>&1 || { echo "fail $v"; exit 1; }
    echo "$v round $round: $(tail -1 gpurun_out/ab/$v.$round.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
