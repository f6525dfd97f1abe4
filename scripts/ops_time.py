"""Setup once (bench settings) and time the big level operators alone (HIP
events, bench_level_op) plus a 10-iteration solve: an A/B tool for layout
switches given through the environment.  python scripts/ops_time.py N"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, "hypre-ve_amd")
import hypreve as hv

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
hv.init()
A = hv.ParCSRMatrix.laplacian(n, n, n)
kw = hv.ij_amg_defaults(0)
kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=18, tol=1e-300, max_iter=10, min_iter=0)
amg = hv.BoomerAMG(**kw)
t = time.time()
amg.setup(A)
row = {"n": n, "env": {k: v for k, v in os.environ.items() if k.startswith("HVE_")}, "setup_s": round(time.time() - t, 1)}
nl = amg.num_levels()
for l, w, name in [(0, 0, "A0"), (0, 1, "P0"), (0, 2, "R0"), (1, 0, "A1"), (1, 1, "P1"), (1, 2, "R1"), (2, 0, "A2"),
                   (2, 1, "P2"), (2, 2, "R2"), (3, 0, "A3"), (3, 1, "P3"), (3, 2, "R3"), (4, 0, "A4")]:
    if l >= nl or (w and l >= nl - 1):
        continue
    ms = amg.bench_level_op(l, w, 20)[0]
    row[name] = [amg.level_layout(l, w), round(ms, 4), round(amg.level_op_stored_bytes(l, w) / ms / 1e6, 0)]
b = hv.ParVector(A.n, np.ones(A.n))
x = hv.ParVector(A.n, np.zeros(A.n))
amg.solve(A, b, x)
x.fill(0.0)
hv.lib().hypreve_DeviceSynchronize()
t = time.perf_counter()
amg.solve(A, b, x)
hv.lib().hypreve_DeviceSynchronize()
row["ms_per_iter"] = round((time.perf_counter() - t) / 10 * 1e3, 3)
print(json.dumps(row), flush=True)
