"""HBM traffic per launch of the finest-level residual SpMV from rocprofv3 PMC
passes over bench.py (one pass FETCH_SIZE, one pass WRITE_SIZE, each with
--kernel-trace only, as MI355X_MICROARCH.md's HBM/rocprofv3 section asks).

Corrections (MI355X_MICROARCH.md, "HBM [CDNA4]"): FETCH_SIZE is in KiB and on
gfx950 reports half the bytes of a streaming read -- checked here for our own
widths with the stream-read calibration kernel (4 B and 8 B per lane both read
back exactly 0.5x); WRITE_SIZE (KiB) is exact.  traffic = 2 * FETCH + WRITE.

    python scripts/pmc_traffic.py <dir with pmc_fetch/ pmc_write/> <grid> [out.json]

grid = Grid_Size of the finest-level launches (256 * blocks, 16777216 at 256^3).
"""
import csv
import json
import os
import sys


PREFIXES = ("hve::k_sell<0,", "hve::k_sell_delta<0,", "hve::k_sell_stencil<0,")


def mean_counter(path, counter, grid, prefixes=PREFIXES, names=None):
    vals = []
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter or (grid is not None and int(r["Grid_Size"]) != grid):
            continue
        nm = r["Kernel_Name"].replace("void ", "")
        if nm.startswith(prefixes):
            vals.append(float(r["Counter_Value"]))
            if names is not None:
                names.add(nm)
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


def stream_calibration(path):
    """FETCH_SIZE (bytes) / bytes read of bench.py --calib's 512 MiB streams."""
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != "FETCH_SIZE":
            continue
        nm = r["Kernel_Name"].replace("void ", "")
        for t, eb in (("short", 2), ("int", 4), ("double", 8)):
            if nm.startswith(f"hve::k_stream_read<{t}>"):
                out.setdefault(f"{eb}B", []).append(float(r["Counter_Value"]) * 1024 / (1 << 29))
    return {k: round(min(v), 4) for k, v in out.items()}


def main():
    root, grid = sys.argv[1], int(sys.argv[2])
    # the cycle's own finest residual kernel: the first layout family with
    # dispatches at this grid (bench.py also times the general padded path,
    # hve::k_sell<0, ...>, on the same grid: it must not be averaged in)
    fpath = os.path.join(root, "pmc_fetch", "run_counter_collection.csv")
    wpath = os.path.join(root, "pmc_write", "run_counter_collection.csv")
    fetch = write = None
    names = set()
    # (the grid-stencil loop launches one workgroup per tile and plane chunk,
    # not per row block: any grid size; only level 0 has the grid layout)
    for pre in ("hve::k_grid_stencil<0,", "hve::k_sell_stencil<0,", "hve::k_sell_delta<0,", "hve::k_sell<0,"):
        names = set()
        g = None if pre.startswith("hve::k_grid") else grid
        fetch, nf = mean_counter(fpath, "FETCH_SIZE", g, prefixes=(pre,), names=names)
        write, nw = mean_counter(wpath, "WRITE_SIZE", g, prefixes=(pre,))
        if fetch is not None and write is not None:
            break
    if fetch is None or write is None:
        raise SystemExit("no matching dispatches")
    out = {"kernel": "k_grid_stencil / k_sell_stencil / k_sell_delta / k_sell <OP_RESID> finest level", "kernel_names": sorted(names),
           "grid": grid, "dispatches": [nf, nw],
           "fetch_kib": fetch, "write_kib": write,
           "traffic_bytes": 2.0 * fetch * 1024 + write * 1024,
           "correction": "traffic = 2*FETCH_SIZE + WRITE_SIZE (KiB->B); FETCH x2 per MI355X_MICROARCH.md, "
                         "checked with the 4/8-B stream calibration kernel",
           "fetch_ratio_of_stream_bytes": stream_calibration(
               os.path.join(root, "pmc_fetch", "run_counter_collection.csv"))}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
