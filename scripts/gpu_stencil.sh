#!/bin/bash
# Stencil-layout checks in one gpurun call: the layout's parity tests, the
# slices-per-wave sweep at 256^3 (ops_time.py), segmented-stream reference.
set -u
mkdir -p gpurun_out
OUT=gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -4 "$OUT/$name.log"
  case $rc in
    0|1|2|5) return 0 ;;
    *) echo "=== stopping after $name (rc=$rc)"; exit $rc ;;
  esac
}
step st_tests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 300 --timeout-method thread -k "policy or stride or bench_size or 27pt or aniso or stencil or partitioned_solve"
step streams 300 python -c "
import sys; sys.path.insert(0,'hypre-ve_amd'); import hypreve as hv; hv.init()
n=(1<<31)//8
for eb,name in ((8,'grid-stride'),(-8,'per-wave 16KiB segments'),(-9,'interleaved 512B chunks')):
    ms=hv.bench_stream(eb,n,10); print(f'{name}: {n*8/(ms*1e-3)/1e9:.0f} GB/s', flush=True)
"
for R in 1 2 4; do
  HVE_STENCIL_R=$R step ops256_R$R 300 python scripts/ops_time.py 256
done
echo "=== done"
