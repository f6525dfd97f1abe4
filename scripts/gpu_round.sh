#!/bin/bash
# One gpurun call: GPU tests, smoke, bench, rocprof profiles.  Every GPU step has
# its own time limit; after a fault / abort / timeout nothing further runs.
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
  tail -5 "$OUT/$name.log"
  case $rc in
    0|1|2|5) return 0 ;;   # pass / test failures / usage: keep going
    *) echo "=== stopping after $name (rc=$rc)"; exit $rc ;;
  esac
}
WHAT=${1:-all}
want() { [[ $WHAT == all || ,$WHAT, == *,$1,* ]]; }  # e.g. tests,share,bench
if want tests; then
  step pytest_gpu 1200 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if want multi; then
  # the driver's multi-GPU launch shape, with one rank: torch.distributed.run,
  # gloo for the unique id and the timing max, a 1-rank RCCL communicator
  step dist1 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 1 --dist --steps 5 --warmup 1 --cpu-cycles 0
fi
if want share; then
  # one rank's share of the 8-GPU strong split of configs[3] / configs[4]
  # (512 x 512 x 64 rows) on a 1-rank RCCL communicator: setup time and RSS
  step share27 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29556 bench.py --gpus 1 --dist --grid 512,512,64 --stencil 27 --steps 10 --warmup 2 --cpu-cycles 0
  step shareagg 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29557 bench.py --gpus 1 --dist --grid 512,512,64 --coef 0.001,1,1 --agg 1 --steps 10 --warmup 2 --cpu-cycles 0
fi
if want loop; then
  step loopback2 600 python bench.py --loopback 2 --n 128 --steps 5 --warmup 1 --cpu-cycles 0
  step loopback8 900 python bench.py --loopback 8 --n ${LOOPBACK_N:-128} --steps 3 --warmup 1 --cpu-cycles 0
fi
if want bench; then
  step bench 900 python bench.py --steps 10 --warmup 2
fi
if want prof; then
  step rocprof_stats 900 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --cpu-cycles 0
fi
echo "=== done"
