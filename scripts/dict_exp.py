"""Timing-only phase experiment on the dictionary loop (k_sell_dict): with the
library built with -DHVE_DICT_EXP (HVE_LIB_PATH), knob 12 leaves out phases
(1 the x-tile gather, 2 the column loads, 4 the value loads; results are then
wrong, times only).  Sets up the bench hierarchy at N^3 once and times A_1,
R_1 and A_2 alone for each combination.  python scripts/dict_exp.py N"""
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
rows = []
for exp in (0, 1, 2, 4, 6, 7, 0):
    hv.set_knob(12, exp)
    row = {"exp": exp}
    for name, (l, w) in (("A1", (1, 0)), ("R1", (1, 2)), ("A2", (2, 0))):
        ms = amg.bench_level_op(l, w, 20)[0]
        sb = amg.level_op_stored_bytes(l, w)
        row[name] = [round(ms, 4), round(sb / (ms * 1e-3) / 1e9, 1)]
    print(json.dumps(row), flush=True)
hv.set_knob(12, 0)
