"""Time selected level operators of the bench hierarchy (for rocprofv3 PMC
passes on one kernel).

    python scripts/op_bench.py [--n 256] [--ops 1A,0R,2A] [--reps 10]

Each op is <level><A|P|R>; runs bench_level_op (residual form for A,
prolongation for P, restriction for R) `reps` times after the setup.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hypre-ve_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--ops", default="1A")
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    import torch  # noqa: F401
    import hypreve as hv

    hv.init()
    A = hv.ParCSRMatrix.laplacian(args.n, args.n, args.n)
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=18)
    amg = hv.BoomerAMG(**kw)
    t = time.time()
    amg.setup(A)
    print(f"setup {time.time()-t:.1f}s", flush=True)
    for op in args.ops.split(","):
        lvl, which = int(op[:-1]), "APR".index(op[-1])
        ms, by, pad = amg.bench_level_op(lvl, which, args.reps)
        print(f"{op}: {ms*1e3:.1f} us, {by/1e9:.3f} GB algorithmic, {by/(ms*1e-3)/1e9:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
