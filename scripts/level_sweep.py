"""Per-level operator timings of the bench hierarchy (256^3 7-point Laplacian,
PMIS + ext+i Pmx 4, relax 18) and read-only stream references.

    python scripts/level_sweep.py [--n 256] [--reps 20]

Prints one line per (level, operator): rows, nnz, SELL padding, avg us,
algorithmic GB/s.  Kernel variants are chosen by environment variables read
by the library (HVE_SELL_BATCH, HVE_SELL_PIPE), so run one process per variant.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hypre-ve_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--coarsen", type=int, default=8)
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    import torch  # noqa: F401  (shares the HIP runtime)
    import hypreve as hv

    hv.init()
    variant = {k: os.environ.get(k, "") for k in ("HVE_SELL_BATCH", "HVE_SELL_PIPE", "HVE_SELL_NT", "HVE_SELL_JAG")}
    print(f"variant {variant}", flush=True)
    rows = []
    for eb in (4, 8, 16):
        n = (1 << 31) // eb  # 2 GiB
        ms = hv.bench_stream(eb, n, args.reps)
        gbs = n * eb / (ms * 1e-3) / 1e9
        print(f"stream read {eb} B/lane: {ms*1e3:.1f} us for {n*eb/2**30:.0f} GiB -> {gbs:.0f} GB/s", flush=True)
        rows.append({"kind": "stream", "elem_bytes": eb, "ms": ms, "gbs": gbs})
    A = hv.ParCSRMatrix.laplacian(args.n, args.n, args.n)
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=args.coarsen, interp_type=6, P_max_elmts=4, relax_type=18)
    amg = hv.BoomerAMG(**kw)
    t = time.time()
    amg.setup(A)
    print(f"setup {time.time()-t:.1f}s levels {amg.num_levels()}", flush=True)
    tot = 0.0
    for l in range(amg.num_levels()):
        r, annz, pnnz = amg.level_info(l)
        for which, name in ((0, "A"), (1, "P"), (2, "R")):
            if which and l == amg.num_levels() - 1:
                continue
            ms, by, pad = amg.bench_level_op(l, which, args.reps)
            nnz = annz if which == 0 else pnnz
            gbs = by / (ms * 1e-3) / 1e9
            print(f"L{l} {name} rows={r if which != 2 else '-':>9} nnz={nnz:>11} pad={pad/max(nnz,1):.3f} "
                  f"{ms*1e3:9.1f} us {gbs:7.0f} GB/s  {amg.level_layout(l, which)}", flush=True)
            rows.append({"kind": "op", "level": l, "op": name, "rows": r, "nnz": nnz, "pad": pad / max(nnz, 1),
                         "us": ms * 1e3, "gbs": gbs})
    if args.json:
        with open(args.json, "w") as f:
            json.dump({"variant": variant, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
