#!/bin/bash
# rocprofv3 PMC passes over solve iterations only (scripts/cycle_trace.py):
# FETCH_SIZE, WRITE_SIZE and TCC hit/miss, each in its own pass, then the
# per-kernel summary and the finest-residual traffic JSON.  N=${N:-512}.
set -u
N=${N:-512}
OUT=gpurun_out/pmccyc$N
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
RUN="scripts/cycle_trace.py $N 3 ${EXTRA:-}"
step pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o run --output-format csv -- python $RUN
step pmc_write 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o run --output-format csv -- python $RUN
step pmc_hit 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $OUT/pmc_hit -o run --output-format csv -- python $RUN
for d in pmc_fetch pmc_write pmc_hit; do
  f=$(find $OUT/$d -mindepth 2 -name run_counter_collection.csv | sort | tail -1); [[ -n $f ]] && cp $f $OUT/$d/run_counter_collection.csv
done
python scripts/pmc_summary.py $OUT 60000 > $OUT/pmc_summary.txt 2>&1
python scripts/pmc_traffic.py $OUT $((N*N*N)) $OUT/pmc_traffic_$N.json > $OUT/pmc_traffic.log 2>&1
echo "=== done"
