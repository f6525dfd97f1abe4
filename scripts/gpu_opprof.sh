#!/bin/bash
# Counter passes over the large level operators at N^3 (scripts/op_pmc.py),
# one rocprofv3 process per counter set (MI355X_MICROARCH.md: no pass
# splitting; block slot limits), then scripts/pmc_ops_table.py joins them.
#   OUT=gpurun_out/x N=512 bash scripts/gpu_opprof.sh
N=${N:-512}
OUT=${OUT:-gpurun_out/opprof$N}
source scripts/gpu_step.sh
OPS=${OPS:-A0,P0,R0,A1,P1,R1,A2}
run() { python scripts/op_pmc.py $N 5 $OPS; }
step trace 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python scripts/op_pmc.py $N 5 $OPS
pass() {  # pass <name> <counters...>
  local name=$1; shift
  step pmc_$name 600 rocprofv3 --pmc "$@" --kernel-trace -d $OUT/pmc_$name -o run --output-format csv -- python scripts/op_pmc.py $N 5 $OPS
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass l2 TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE
pass ta TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum
python scripts/pmc_ops_table.py $OUT > $OUT/pmc_ops_table.txt 2>&1
echo "=== done"
