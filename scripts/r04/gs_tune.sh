#!/bin/bash
# GS cycle at N^3 for several team sizes / gather orders / library builds
# (variant T:TW:NAT[:LIB], a kernel trace per variant).
set -u
OUT=gpurun_out/${TAG:-gs_tune}
mkdir -p $OUT
export TMPDIR=/tmp
for V in ${VARIANTS:-"64:16:0"}; do
  IFS=: read T TW NAT LIB <<< "$V"
  NAME=$T-$TW-$NAT-$(basename ${LIB:-lib})
  HVE_LIB_PATH=${LIB:-hypre-ve_amd/lib/libhypreve.so} HVE_GS_TEAM_ROWS=$T HVE_GS_TEAM_ROWS_WIDE=$TW HVE_GS_NAT=$NAT \
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace_$NAME -o run --output-format csv -- \
    python bench.py --n ${N:-256} --secondary-n 0 --cpu-cycles 0 --relax -1 --steps 10 --warmup 2 --spmv-reps 5 \
    > $OUT/bench_$NAME.log 2>&1 || { tail -20 $OUT/bench_$NAME.log; exit 1; }
  echo "== $V: $(grep 'steps in' $OUT/bench_$NAME.log)"
done
