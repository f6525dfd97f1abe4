#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over scripts/op_bench.py.
set -u
OUT=gpurun_out/pmcops
mkdir -p $OUT
export TMPDIR=/tmp
OPS=${OPS:-1A,0R,2A,0A}
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" "SQ_WAVES SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_WAVE_CYCLES SQ_INSTS_VALU" "TCC_HIT_sum TCC_MISS_sum" "TD_BUSY_avr TD_TC_STALL_sum"; do
  i=$((i+1))
  echo "=== pass $i: $grp"
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d $OUT/p$i -o run --output-format csv -- python scripts/op_bench.py --ops $OPS --reps 5 > $OUT/p$i.log 2>&1
  rc=$?
  echo "rc=$rc"; tail -2 $OUT/p$i.log
  if [ $rc -ne 0 ]; then echo "stopping"; break; fi
done
