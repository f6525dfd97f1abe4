"""Per-operator times on one rank's share of an 8-GPU workload (one GPU, no
communicator): configs[4] by default (anisotropic 0.001,1,1 on 512x512x64,
PMIS + 1 aggressive level).  Layout variants are chosen by the library's
environment switches (HVE_SELL_DICT, HVE_SELL_JAG, HVE_SELL_WIDE_ROWS, ...),
one process per variant.
    python scripts/share_ops.py [--grid 512,512,64] [--coef 0.001,1,1] [--agg 1] [--stencil 7]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "hypre-ve_amd"))
import hypreve as hv  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", default="512,512,64")
    ap.add_argument("--coef", default="0.001,1,1")
    ap.add_argument("--agg", type=int, default=1)
    ap.add_argument("--stencil", type=int, default=7)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    nx, ny, nz = (int(v) for v in a.grid.split(","))
    cx, cy, cz = (float(v) for v in a.coef.split(","))
    hv.init()
    A = (hv.ParCSRMatrix.laplacian27(nx, ny, nz) if a.stencil == 27
         else hv.ParCSRMatrix.laplacian(nx, ny, nz, cx=cx, cy=cy, cz=cz))
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=18, agg_num_levels=a.agg, tol=1e-300,
              max_iter=20, min_iter=0)
    amg = hv.BoomerAMG(**kw)
    t = time.time()
    amg.setup(A)
    row = {"env": {k: v for k, v in os.environ.items() if k.startswith("HVE_")}, "setup_s": round(time.time() - t, 1)}
    nl = amg.num_levels()
    for l in range(min(nl, 4)):
        for w, nm in ((0, "A"), (1, "P"), (2, "R")):
            if w and l >= nl - 1:
                continue
            ms = amg.bench_level_op(l, w, a.reps)[0]
            sb = amg.level_op_stored_bytes(l, w)
            r, annz, pnnz = amg.level_info(l)
            row[f"{nm}{l}"] = [amg.level_layout(l, w), round(ms, 4), round(sb / (ms * 1e-3) / 8e12, 3),
                               r, annz if w == 0 else pnnz]
    b = hv.ParVector(A.n, np.ones(A.n))
    x = hv.ParVector(A.n, np.zeros(A.n))
    amg.solve(A, b, x)
    x.fill(0.0)
    hv.lib().hypreve_DeviceSynchronize()
    t = time.perf_counter()
    amg.solve(A, b, x)
    hv.lib().hypreve_DeviceSynchronize()
    row["ms_per_step"] = round((time.perf_counter() - t) / 20 * 1e3, 4)
    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
