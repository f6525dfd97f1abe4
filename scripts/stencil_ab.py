"""A/B of the finest-level stencil kernels alone (hypreve_BenchOperator): the
7-point (and optionally 27-point) operator at n^3 uploaded in its automatic
layout with the bench's traversal, ops residual / l1-Jacobi / fused residual +
l1-Jacobi timed with HIP events.  Kernel variants are chosen through HVE_*
environment variables by the caller (one process per variant).

    python scripts/stencil_ab.py [--n 512] [--stencil 7] [--reps 30] [--tag name]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hypre-ve_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--stencil", type=int, default=7)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--bands", type=int, default=8)
    ap.add_argument("--tag", default="")
    ap.add_argument("--settings", default="", help="knob settings 'k=v,k=v;k=v' (hypreve_SetKnob), one row each")
    args = ap.parse_args()
    import torch  # noqa: F401
    import hypreve as hv

    hv.init()
    t = time.time()
    n = args.n
    A = hv.ParCSRMatrix.laplacian27(n, n, n) if args.stencil == 27 else hv.ParCSRMatrix.laplacian(n, n, n)
    base = {"tag": args.tag, "n": n, "stencil": args.stencil,
            "env": {k: v for k, v in os.environ.items() if k.startswith("HVE_")}, "gen_s": round(time.time() - t, 1)}
    for st in args.settings.split(";"):
        knobs = dict((int(a), int(b)) for a, b in (kv.split("=") for kv in filter(None, st.split(","))))
        for k in range(16):
            hv.set_knob(k, knobs.get(k, 0))
        row = dict(base, knobs=knobs)
        for op, name in ((0, "resid"), (2, "l1jac"), (8, "resid_l1jac")):
            t = time.time()
            ms, by, lay = A.bench_operator(op=op, policy=0, nbands=args.bands, reps=args.reps)
            row[name] = {"ms": round(ms, 4), "GBs": round(by / ms / 1e6, 1), "frac": round(by / ms / 1e6 / 8000, 4)}
            row["layout"] = lay
            row["upload_s"] = round(time.time() - t, 1)
        print(json.dumps(row), flush=True)
    A.destroy()


if __name__ == "__main__":
    main()
