#!/bin/bash
# A1 dictionary-loop bottleneck experiments at 256^3 (ops_time.py per variant)
set -u
mkdir -p gpurun_out/exp
OUT=gpurun_out/exp
export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$OUT/$name.log"
  case $rc in 0|1|2|5) return 0 ;; *) echo "=== stopping after $name (rc=$rc)"; exit $rc ;; esac
}
step streams 300 python -c "
import sys; sys.path.insert(0,'hypre-ve_amd'); import hypreve as hv; hv.init()
n=(1<<31)//8
for eb,name in ((8,'grid-stride'),(-8,'per-wave 16KiB segments'),(-9,'interleaved 512B chunks')):
    ms=hv.bench_stream(eb,n,10); print(f'{name}: {n*8/(ms*1e-3)/1e9:.0f} GB/s', flush=True)
m=1<<27
for R in (1,2,5):
    ms=hv.bench_stream(-R,m,10); print(f'mix {R} read + 1 write: {m*8*(R+1)/(ms*1e-3)/1e9:.0f} GB/s', flush=True)
"
step base 300 python scripts/ops_time.py 256
HVE_EXPER=1 step nogather 300 python scripts/ops_time.py 256
HVE_EXPER=3 step nogather_nolds 300 python scripts/ops_time.py 256
HVE_EXPER=2 step nolds 300 python scripts/ops_time.py 256
HVE_SELL_BATCH=8 step batch8 300 python scripts/ops_time.py 256
echo "=== done"
