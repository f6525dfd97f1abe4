"""Per-operator traversal bands (tuning): one setup, then for each operator
class (A, P, R) and band count, that class's big operators timed alone.
python scripts/band_op_sweep.py N [bands]"""
import json
import sys
import time

sys.path.insert(0, "hypre-ve_amd")
import hypreve as hv

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
bands = [int(b) for b in (sys.argv[2] if len(sys.argv) > 2 else "0,8,16,32,64,128").split(",")]
hv.init()
A = hv.ParCSRMatrix.laplacian(n, n, n)
kw = hv.ij_amg_defaults(0)
kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=18)
amg = hv.BoomerAMG(**kw)
t = time.time()
amg.setup(A)
print(f"setup {time.time() - t:.1f}s", flush=True)
ops = {"A": [(0, 0, "A0"), (1, 0, "A1"), (2, 0, "A2")], "P": [(0, 1, "P0"), (1, 1, "P1")],
       "R": [(0, 2, "R0"), (1, 2, "R1")]}
for cls, lst in ops.items():
    for nb in bands:
        amg.set_block_bands(nb, cls)
        row = {"class": cls, "bands": nb}
        for l, w, name in lst:
            row[name] = round(amg.bench_level_op(l, w, 20)[0], 4)
        print(json.dumps(row), flush=True)
    amg.set_block_bands(8, cls)
