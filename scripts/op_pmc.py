"""Set up the bench hierarchy once (PMIS, ext+i Pmx 4, relax 18) and apply the
large level operators alone, `reps` times each (hypreve_BenchLevelOp): the
process that rocprofv3 --pmc passes run, one counter set per process
(scripts/gpu_opprof.sh).  python scripts/op_pmc.py N [reps] [ops]"""
import json
import sys
import time

sys.path.insert(0, "hypre-ve_amd")
import hypreve as hv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
ops = sys.argv[3].split(",") if len(sys.argv) > 3 else ["A0", "P0", "R0", "A1", "P1", "R1", "A2"]
hv.init()
A = hv.ParCSRMatrix.laplacian(n, n, n)
kw = hv.ij_amg_defaults(0)
kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=18)
amg = hv.BoomerAMG(**kw)
t = time.time()
amg.setup(A)
print(f"setup {time.time() - t:.1f}s", flush=True)
where = {"A0": (0, 0), "P0": (0, 1), "R0": (0, 2), "A1": (1, 0), "P1": (1, 1), "R1": (1, 2), "A2": (2, 0),
         "P2": (2, 1), "R2": (2, 2)}
row = {"n": n}
for name in ops:
    l, w = where[name]
    ms = amg.bench_level_op(l, w, reps)[0]
    sb = amg.level_op_stored_bytes(l, w)
    row[name] = {"layout": amg.level_layout(l, w), "ms": round(ms, 4), "stored_bytes": sb,
                 "frac": round(sb / (ms * 1e-3) / 8e12, 4)}
    print(name, row[name], flush=True)
print(json.dumps(row), flush=True)
