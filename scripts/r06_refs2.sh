# configs[4] at 512^3 (its N = 1 line: column 1 of the digests) and the
# one-GPU references of its 2 / 4 / 8-rank lines; the 27-point operator's at
# 256^3 (r06_refs.sh), each step under its own time limit.
bash_step() { "$@" || { echo "exit $?"; exit 1; }; }
mkdir -p gpurun_out/r06/08_refs_cfg
bash_step timeout -k 10 600 python -u bench.py --coef 0.001,1,1 --agg 1 --steps 10 --warmup 2 --secondary-n 0 --setup-parity 0 --pcg-iters 0 --gs-n 0 > gpurun_out/r06/08_refs_cfg/agg512.txt 2>&1
REF_TIMEOUT=300 bash scripts/r06_refs.sh 08_refs_cfg/agg "--n 512 --coef 0.001,1,1 --agg 1" 2 4 8 | tail -1 | grep -q "exit 0" || { echo "exit 1"; exit 1; }
REF_TIMEOUT=200 bash scripts/r06_refs.sh 08_refs_cfg/s27 "--n 256 --stencil 27" 2 4 8
