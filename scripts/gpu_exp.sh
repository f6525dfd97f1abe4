#!/bin/bash
# Kernel-variant sweep and PMC counter passes (one gpurun call).  Each GPU step
# has its own time limit; after a fault / abort / timeout nothing further runs.
set -u
mkdir -p gpurun_out/exp
OUT=gpurun_out/exp
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -3 "$OUT/$name.log"
  case $rc in
    0|1|2|5) return 0 ;;
    *) echo "=== stopping after $name (rc=$rc)"; exit $rc ;;
  esac
}
WHAT=${1:-all}
if [[ $WHAT == all || $WHAT == tests ]]; then
  step pytest_gpu 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
fi
if [[ $WHAT == all || $WHAT == sweep ]]; then
  # default layout choice against forced variants (env read by the library)
  step sweep_auto 300 python scripts/level_sweep.py --json $OUT/sweep_auto.json
  step bench 600 python bench.py --steps 10 --warmup 2 --cpu-cycles 0
  for v in ${SWEEP_VARIANTS:-HVE_SELL_JAG=0}; do
    timeout -k 10 300 env ${v//,/ } python scripts/level_sweep.py --json $OUT/sweep_$v.json > $OUT/sweep_$v.log 2>&1 || exit 1
    tail -2 $OUT/sweep_$v.log
  done
fi
if [[ $WHAT == all || $WHAT == pmc ]]; then
  step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --cpu-cycles 0 --spmv-reps 5 --calib
  step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --cpu-cycles 0 --spmv-reps 5
  step pmc_tcc 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $OUT/pmc_tcc -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --cpu-cycles 0 --spmv-reps 5
  python scripts/pmc_traffic.py $OUT 16777216 $OUT/pmc_traffic_256.json > $OUT/pmc_traffic.log 2>&1
  python scripts/pmc_summary.py $OUT 60000 > $OUT/pmc_summary.txt 2>&1
fi
echo "=== done"
