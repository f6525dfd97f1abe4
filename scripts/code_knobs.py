"""Coded-loop launch knobs (knob 0: rows per lane, 1: codes per batch, 2:
workgroups per CU) swept on R_0 and P_0 of the bench hierarchy at N^3, each
timed alone (HIP events, bench_level_op).  python scripts/code_knobs.py N"""
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
for nr, cb, wpc in [(1, 8, 8), (2, 8, 8), (2, 4, 8), (4, 4, 8), (1, 4, 8), (1, 16, 8), (1, 8, 4), (1, 8, 16), (2, 8, 4)]:
    hv.set_knob(0, nr)
    hv.set_knob(1, cb)
    hv.set_knob(2, wpc)
    row = {"nr": nr, "cb": cb, "wpc": wpc}
    for name, (l, w) in (("R0", (0, 2)), ("P0", (0, 1))):
        ms = amg.bench_level_op(l, w, 20)[0]
        row[name] = [round(ms, 4), round(amg.level_op_stored_bytes(l, w) / (ms * 1e-3) / 1e9, 1)]
    print(json.dumps(row), flush=True)
for k in (0, 1, 2):
    hv.set_knob(k, 0)
