"""R_0 on the jagged product-parallel coded loop (sell policy 15 at upload):
knob 4 = entries per row and chunk (4 | 8 | 16), knob 5 = 1 turns the code
prefetch off, knob 2 caps workgroups per CU; each variant timed alone on the
bench hierarchy at N^3 (HIP events, bench_level_op).  Without "jag" the
padded coded loop's time is printed for comparison.
python scripts/r0_pw_knobs.py N [jag]"""
import json
import sys

sys.path.insert(0, "hypre-ve_amd")
import hypreve as hv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
hv.init()
A = hv.ParCSRMatrix.laplacian(n, n, n)
kw = hv.ij_amg_defaults(0)
kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=18)
jag = "jag" in sys.argv[2:]
if jag:
    kw.update(sell_policy=15)
amg = hv.BoomerAMG(**kw)
amg.setup(A)
layout = amg.level_layout(0, 2)
variants = [(8, 0, 4), (8, 1, 4), (8, 0, 3), (8, 1, 3), (8, 0, 2), (8, 1, 2), (4, 0, 4), (4, 0, 2), (8, 0, 6), (8, 0, 4)]
if not jag:
    variants = [(0, 0, 0), (0, 0, 6), (0, 0, 4), (0, 0, 3), (0, 0, 0)]
for kc, nopf, wpc in variants:
    hv.set_knob(4, kc)
    hv.set_knob(5, nopf)
    hv.set_knob(2, wpc)
    ms = amg.bench_level_op(0, 2, 30)[0]
    gbs = amg.level_op_stored_bytes(0, 2) / (ms * 1e-3) / 1e9
    print(json.dumps({"layout": layout, "kc": kc, "prefetch": nopf != 1, "wpc": wpc,
                      "R0_ms": round(ms, 4), "GB/s": round(gbs, 1)}), flush=True)
for k in (2, 4, 5):
    hv.set_knob(k, 0)
