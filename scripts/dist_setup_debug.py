"""Run the distributed-setup self-check for one configuration (CPU only; for
debugging a failing parametrisation of tests/test_setup_host.py under gdb).

    python scripts/dist_setup_debug.py <ranks> [relax] [order] [cy]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hypre-ve_amd"))
import hypreve as hv  # noqa: E402

size = int(sys.argv[1])
relax = int(sys.argv[2]) if len(sys.argv) > 2 else 0
order = int(sys.argv[3]) if len(sys.argv) > 3 else 1
cy = float(sys.argv[4]) if len(sys.argv) > 4 else 0.7
A = hv.ParCSRMatrix.laplacian(19, 17, 23, cx=1.0, cy=cy, cz=1.0)
amg = hv.BoomerAMG(**hv.ij_amg_defaults(0))
amg.set(coarsen_type=8, interp_type=6, relax_type=relax, relax_order=order, P_max_elmts=4)
amg.dist_setup_check(A, size)
print("ok")
