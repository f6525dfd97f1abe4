#!/bin/bash
OUT=gpurun_out/r05o
source scripts/gpu_step.sh
B="python -u bench.py --relax -1 --n 256 --secondary-n 0 --setup-parity 0 --pcg-iters 0 --steps 3 --warmup 1 --cpu-cycles 0 --spmv-reps 1"
step trace 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B
pass() {
  local name=$1; shift
  step pmc_$name 300 rocprofv3 --pmc "$@" --kernel-trace -d $OUT/pmc_$name -o run --output-format csv -- $B
}
pass fetch FETCH_SIZE
pass l2 TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE
pass sq2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
pass ta TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum
python scripts/pmc_ops_table.py $OUT > $OUT/pmc_ops_table.txt 2>&1
echo "=== done"
