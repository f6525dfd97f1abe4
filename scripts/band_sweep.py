"""Row-block traversal sweep (one setup): per band count, the big operators
timed alone (HIP events) and a 10-iteration solve.  Tuning tool."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, "hypre-ve_amd")
import hypreve as hv

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
bands = [int(b) for b in (sys.argv[2] if len(sys.argv) > 2 else "0,8,16,32,64,128").split(",")]
hv.init()
A = hv.ParCSRMatrix.laplacian(n, n, n)
kw = hv.ij_amg_defaults(0)
kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=18, tol=1e-300, max_iter=10, min_iter=0)
amg = hv.BoomerAMG(**kw)
t = time.time()
amg.setup(A)
print(f"setup {time.time() - t:.1f}s", flush=True)
b = hv.ParVector(A.n, np.ones(A.n))
x = hv.ParVector(A.n, np.zeros(A.n))
ops = [(0, 0, "A0"), (0, 1, "P0"), (0, 2, "R0"), (1, 0, "A1"), (1, 2, "R1"), (2, 0, "A2")]
for nb in bands:
    amg.set_block_bands(nb)
    row = {"bands": nb}
    for l, w, name in ops:
        row[name] = round(amg.bench_level_op(l, w, 20)[0], 4)
    amg.solve(A, b, x)
    x.fill(0.0)
    hv.lib().hypreve_DeviceSynchronize()
    t = time.perf_counter()
    amg.solve(A, b, x)
    hv.lib().hypreve_DeviceSynchronize()
    row["ms_per_iter"] = round((time.perf_counter() - t) / 10 * 1e3, 3)
    x.fill(0.0)
    print(json.dumps(row), flush=True)
