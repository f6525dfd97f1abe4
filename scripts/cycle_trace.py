"""Solve iterations only (no per-kernel benches), for a per-step kernel
breakdown under rocprofv3 --kernel-trace:  python scripts/cycle_trace.py N ITERS.
Settings as bench.py's V-cycle line.  Per-step times: trace_summary.py totals
divided by ITERS + 1 (one warm-up solve iteration)."""
import sys
import time

import numpy as np

sys.path.insert(0, "hypre-ve_amd")
import hypreve as hv

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
extra = dict(kv.split("=") for kv in sys.argv[3:])
hv.init()
A = hv.ParCSRMatrix.laplacian(n, n, n)
kw = hv.ij_amg_defaults(0)
kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=18, tol=1e-300, max_iter=1, min_iter=0)
kw.update({k: type(kw.get(k, 0))(float(v)) if k in kw else int(v) for k, v in extra.items()})
if kw["relax_type"] < 0:  # relax_type=-1: BoomerAMG's default smoothers (hybrid GS 13 / 14)
    del kw["relax_type"]
amg = hv.BoomerAMG(**kw)
t = time.time()
amg.setup(A)
print(f"setup {time.time() - t:.1f}s levels {amg.num_levels()}", flush=True)
b = hv.ParVector(A.n, np.ones(A.n))
x = hv.ParVector(A.n, np.zeros(A.n))
amg.solve(A, b, x)  # warm-up (graph capture)
amg.set(max_iter=iters)
hv.lib().hypreve_DeviceSynchronize()
t = time.perf_counter()
amg.solve(A, b, x)
hv.lib().hypreve_DeviceSynchronize()
print(f"{iters} iterations: {(time.perf_counter() - t) / iters * 1e3:.3f} ms/iter", flush=True)
