"""Setup time of the bench hierarchy split into the host phases (the setup log:
strength, coarsening, interpolation, RAP, transpose) and the rest (l1 norms,
device layouts and upload).  python scripts/setup_phases.py N"""
import sys
import time

sys.path.insert(0, "hypre-ve_amd")
import hypreve as hv

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
hv.init()
t = time.time()
A = hv.ParCSRMatrix.laplacian(n, n, n)
print(f"generate {time.time() - t:.1f}s", flush=True)
kw = hv.ij_amg_defaults(0)
kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=18, print_level=1)
amg = hv.BoomerAMG(**kw)
t = time.time()
amg.setup(A)
print(f"setup total {time.time() - t:.1f}s", flush=True)
