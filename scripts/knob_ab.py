"""Setup once and time level operators under launch-time knob settings
(hypreve_SetKnob), one JSON line per setting: an in-process A/B of kernel
variants on one hierarchy.
    python scripts/knob_ab.py N 'ops' 'k0=v0,k1=v1;k0=...'   (ops e.g. P0,R0)"""
import json
import sys
import time

sys.path.insert(0, "hypre-ve_amd")
import hypreve as hv

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
ops = (sys.argv[2] if len(sys.argv) > 2 else "P0,R0").split(",")
settings = [s for s in (sys.argv[3] if len(sys.argv) > 3 else "").split(";")]
hv.init()
A = hv.ParCSRMatrix.laplacian(n, n, n)
kw = hv.ij_amg_defaults(0)
kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=18, tol=1e-300, max_iter=10, min_iter=0)
amg = hv.BoomerAMG(**kw)
t = time.time()
amg.setup(A)
print(json.dumps({"n": n, "setup_s": round(time.time() - t, 1)}), flush=True)
which = {"A": 0, "P": 1, "R": 2, "J": 3}  # J: A as the l1-Jacobi sweep
for st in settings:
    knobs = {}
    for kv in filter(None, st.split(",")):
        k, v = kv.split("=")
        knobs[int(k)] = int(v)
    for k in range(16):
        hv.set_knob(k, knobs.get(k, 0))
    row = {"knobs": knobs}
    for name in ops:
        l, w = int(name[1:]), which[name[0]]
        ms = min(amg.bench_level_op(l, w, 20)[0] for _ in range(2))
        row[name] = [amg.level_layout(l, w if w < 3 else 0), round(ms, 4),
                     round(amg.level_op_stored_bytes(l, w) / ms / 1e6, 0)]
    print(json.dumps(row), flush=True)
