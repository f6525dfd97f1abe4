"""A_1, R_1, A_2 on the lane-packed dictionary loop with fewer workgroups a CU
(knob 17: extra LDS a workgroup, KiB), each timed alone on the bench
hierarchy at N^3 (HIP events, bench_level_op).  python scripts/dict_occ.py N"""
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
for extra in (0, 8, 16, 32, 56, 0):
    hv.set_knob(17, extra)
    row = {"extra_kib": extra}
    for name, (l, w) in (("A1", (1, 0)), ("R1", (0, 2)), ("A2", (2, 0))):
        if name == "R1":
            l, w = 1, 2
        ms = amg.bench_level_op(l, w, 20)[0]
        row[name] = [amg.level_layout(l, w), round(ms, 4)]
    print(json.dumps(row), flush=True)
hv.set_knob(17, 0)
