#!/bin/bash
# rocprofv3 passes over the default bench (one gpurun call): kernel trace +
# stats, then FETCH_SIZE and WRITE_SIZE in their own passes (MI355X_MICROARCH.md
# HBM section), joined into pmc_traffic_<n>.json.  N=${N:-512}.
set -u
N=${N:-512}
OUT=gpurun_out/prof$N
mkdir -p $OUT
export TMPDIR=/tmp
GRID=$((N*N*N))
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
BENCH="bench.py --n $N --secondary-n 0 --cpu-cycles 0 --pcg-iters 0 --setup-parity 0"
WHAT=${1:-all}
if [[ $WHAT == all || $WHAT == trace ]]; then
  step trace 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python $BENCH --steps 10 --warmup 2
  f=$(find $OUT/trace -name run_kernel_trace.csv | sort | tail -1)
  [[ -n $f ]] && python scripts/trace_summary.py $f 5 > $OUT/trace_summary.txt 2>&1
  s=$(find $OUT/trace -name run_kernel_stats.csv | sort | tail -1)
  [[ -n $s ]] && cp $s $OUT/rocprof_kernel_stats.csv
fi
if [[ $WHAT == all || $WHAT == pmc ]]; then
  step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o run --output-format csv -- python $BENCH --steps 3 --warmup 1 --spmv-reps 5
  step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o run --output-format csv -- python $BENCH --steps 3 --warmup 1 --spmv-reps 5
  for d in pmc_fetch pmc_write; do
    f=$(find $OUT/$d -mindepth 2 -name run_counter_collection.csv | sort | tail -1); [[ -n $f ]] && cp $f $OUT/$d/run_counter_collection.csv
  done
  python scripts/pmc_traffic.py $OUT $GRID $OUT/pmc_traffic_$N.json > $OUT/pmc_traffic.log 2>&1
  python scripts/pmc_summary.py $OUT 60000 > $OUT/pmc_summary.txt 2>&1
fi
echo "=== done"
if [[ $WHAT == rsweep ]]; then
  for R in 2 4; do
    HVE_STENCIL_R=$R step ops${N}_R$R 500 python scripts/ops_time.py $N
  done
fi
