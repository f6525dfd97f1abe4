#!/bin/bash
# PMC counters of the fused residual + restriction kernel (256^3 bench, HVE_FUSE_RR=1).
set -u
OUT=gpurun_out/${TAG:-fused_pmc}
mkdir -p $OUT
export TMPDIR=/tmp
HVE_FUSE_RR=1 timeout -s KILL 240 rocprofv3 --pmc ${PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAVE_CYCLES} \
  --kernel-trace -d $OUT/pmc -o run --output-format csv -- \
  python bench.py --n 256 --secondary-n 0 --cpu-cycles 0 --steps 3 --warmup 1 --spmv-reps 2 > $OUT/pmc.log 2>&1 \
  || { tail -20 $OUT/pmc.log; exit 1; }
f=$(find $OUT/pmc -name run_counter_collection.csv | sort | tail -1)
python - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"][:50]
    if "resid_restrict" not in k and "k_sell_stencil<0" not in k and "k_sell_code<6" not in k: continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); cnt[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    print(k, {c: round(v / max(1, cnt[(k, c)]), 1) for c, v in d.items()})
PY
