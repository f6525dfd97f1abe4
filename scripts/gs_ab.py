"""Hybrid-GS cycle (relax 13 / 14, BoomerAMG's default smoothers) at N^3 under
launch variants, on one hierarchy in one process: knob 6 = 1 unpaired entry
loads, knob 8 = 1 the pipelined sweep on every level (2: on none), knob 10 its
unit capacity, knob 12 = 256 the unpipelined sweep's 256-entry chunks, knob
13 = 1 the separate scatter pass after the sweep.  The
iterates after 4 iterations from x = 0 must be bitwise equal across variants;
then ms per solve iteration, each variant twice.  "rw16": the wide
operators' schedules built with 16-lane ring slots (knob 14 at setup); "quick":
the default launch only; "occ": extra LDS a workgroup (knob 16, fewer
workgroups a CU).  python scripts/gs_ab.py N [rw16] [quick | occ]"""
import hashlib
import json
import sys
import time

import numpy as np

sys.path.insert(0, "hypre-ve_amd")
import hypreve as hv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
iters = 20
VARIANTS = {  # name: {knob: value}
    "default": {},
    "chunk256": {12: 256},
    "unpaired": {6: 1},
    "pipe_auto": {8: 1},
    "scatter": {13: 1},
}
KNOBS = (6, 8, 10, 12, 13, 16)
if "quick" in sys.argv[2:]:  # the default launch only (the ring-width A/B)
    VARIANTS = {"default": {}}
if "occ" in sys.argv[2:]:  # fewer workgroups a CU through extra LDS (knob 16, KiB)
    VARIANTS = {"default": {}, "nopad": {16: -1}, "lds+16": {16: 16}}


def use(v):
    for k in KNOBS:
        hv.set_knob(k, VARIANTS[v].get(k, 0))


hv.init()
rw16 = "rw16" in sys.argv[2:]
hv.set_knob(14, 16 if rw16 else 0)
A = hv.ParCSRMatrix.laplacian(n, n, n)
kw = hv.ij_amg_defaults(0)
kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, tol=1e-300, max_iter=4, min_iter=0)
amg = hv.BoomerAMG(**kw)
t = time.time()
amg.setup(A)
hv.set_knob(14, 0)
print(f"setup {time.time() - t:.1f}s levels {amg.num_levels()} ring16 {rw16}", flush=True)
keep = []  # vectors stay alive: a freed buffer's address could bring back a captured graph
ref = None
for v in VARIANTS:
    use(v)
    b = hv.ParVector(A.n, np.ones(A.n))
    x = hv.ParVector(A.n, np.zeros(A.n))
    keep += [b, x]
    amg.set(max_iter=4)
    amg.solve(A, b, x)
    xv = x.get()
    if ref is None:
        ref = xv
    print(json.dumps({"n": n, "variant": v, "rw16": rw16, "bitwise_equal_default": bool(np.array_equal(xv, ref)),
                      "sha": hashlib.sha256(xv.tobytes()).hexdigest()[:16]}), flush=True)
for rep in range(2):
    for v in VARIANTS:
        use(v)
        b = hv.ParVector(A.n, np.ones(A.n))
        x = hv.ParVector(A.n, np.zeros(A.n))
        keep += [b, x]
        amg.set(max_iter=1)
        amg.solve(A, b, x)  # capture
        amg.set(max_iter=iters)
        hv.lib().hypreve_DeviceSynchronize()
        t = time.perf_counter()
        amg.solve(A, b, x)
        hv.lib().hypreve_DeviceSynchronize()
        ms = (time.perf_counter() - t) / iters * 1e3
        print(json.dumps({"n": n, "variant": v, "rw16": rw16, "ms_per_iter": round(ms, 3)}), flush=True)
use("default")
