"""Coded-loop workgroups a CU (knob 2) on R_0 and P_0 of the bench hierarchy
at N^3, each timed alone (HIP events, bench_level_op), alternating.
python scripts/code_wpc.py N"""
import json
import sys

sys.path.insert(0, "hypre-ve_amd")
import hypreve as hv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
hv.init()
A = hv.ParCSRMatrix.laplacian(n, n, n)
kw = hv.ij_amg_defaults(0)
kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=18)
amg = hv.BoomerAMG(**kw)
amg.setup(A)
for rep in range(2):
    for wpc in (0, 12, 16, 20):
        hv.set_knob(2, wpc)
        row = {"wpc": wpc or 8}
        for name, (l, w) in (("R0", (0, 2)), ("P0", (0, 1))):
            row[name] = round(amg.bench_level_op(l, w, 30)[0], 4)
        print(json.dumps(row), flush=True)
hv.set_knob(2, 0)
