#!/bin/bash
# A/B end-to-end bench on one box: bench.py under each env variant.
# Usage: VARIANTS="X=0 Y=1,Z=2" N=512 ROUNDS=1 bash scripts/ab_bench.sh [steps]
set -u
mkdir -p gpurun_out/ab
STEPS=${1:-20}
N=${N:-512}
ROUNDS=${ROUNDS:-1}
for round in $(seq 1 $ROUNDS); do
  for v in base ${VARIANTS}; do
    e=""; [[ $v != base ]] && e=${v//,/ }
    timeout -k 10 400 env $e python bench.py --n $N --secondary-n 0 --steps $STEPS --warmup 3 --cpu-cycles 0 \
      --spmv-reps 10 > gpurun_out/ab/$v.$N.$round.log 2>&1 || { echo "fail $v"; exit 1; }
    echo "$v n=$N round $round: $(tail -1 gpurun_out/ab/$v.$N.$round.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], [(k["op"], k["avg_ms"]) for k in d["roofline"]["per_kernel"]])')"
  done
done
