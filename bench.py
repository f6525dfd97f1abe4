"""BoomerAMG V-cycle throughput on MI355X (BASELINE.json metric).

Workload: 3-D 7-point Laplacian 512^3 (configs[2]'s grid, the north-star
size), BoomerAMG with PMIS coarsening, extended+i interpolation (P_max_elmts
4), l1-Jacobi down/up smoothing, Gaussian elimination on the coarsest level.
On one GPU the 256^3 problem (configs[1]) is measured after it into
"secondary", and the CPU oracle's iterate after its sample is compared with
the GPU's bit for bit ("parity").
A step = one BoomerAMG solve iteration (hypre_BoomerAMGSolve loop body): one
V-cycle plus the fine-grid residual and its norm.  Inputs are resident in HBM
before the timed region; the host setup phase is not timed.

Multi-GPU: one process per GPU (torch.distributed.run).  Strong scaling by
default: the global 512^3 problem (ij -n is the global size, ij.c:1780) in
z-slab row blocks, as configs[3]/[4] state it; --weak keeps n^3 rows per GPU.
configs[3]: --stencil 27; configs[4]: --coef 0.001,1,1 --agg 1.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "hypre-ve_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


PROFILE_DIR = os.path.join(ROOT, "profiles")


# hypreve_BoomerAMGGetLevelLayout name -> (residual kernel instantiation as
# rocprofv3 names it, minus the batch width: "<prefix>B<suffix>"; description)
KERNEL_OF_LAYOUT = {
    "grid-stencil": ("k_grid_stencil<0, true, |>(hve::SpArgs)",
                     "slot-uniform SELL-64 over the grid, x staged in an LDS ring of tile planes "
                     "(nothing stored per entry)"),
    "stencil": ("k_sell_stencil<0, false, true, |>(hve::SpArgs)",
                "slot-uniform SELL-64 (per slice and slot one column offset, one value and a lane mask; "
                "nothing stored per entry)"),
    "delta+vt8": ("k_sell_delta<0, false, |, true, 1>(hve::SpArgs)",
                  "SELL-64 with 16-bit column deltas and an 8-bit value table"),
    "delta+vt16": ("k_sell_delta<0, false, |, true, 2>(hve::SpArgs)",
                   "SELL-64 with 16-bit column deltas and a 16-bit value table"),
    "delta": ("k_sell_delta<0, false, |, true, 0>(hve::SpArgs)", "SELL-64 with 16-bit column deltas"),
    "dict": ("k_sell_dict<0, false, |, true, ", "jagged SELL-64 with an LDS x-tile dictionary"),
    "dict-ranges": ("k_sell_dict<0, false, |, true, ", "jagged SELL-64 with an LDS x-tile of column ranges"),
    "coded-jag": ("k_code_pw<0, ", "offset-coded rows, jagged, product-parallel"),
    "dict-wide": ("k_sell_dictw<0, false, true, ", "jagged SELL-64 with an LDS x-tile dictionary, lane-packed "
                  "value / column streams"),
    "padded": ("k_sell<0, false, |, ", "padded SELL-64"),
    "jagged": ("k_sell<0, false, |, ", "jagged SELL-64"),
    "wide": ("k_sell_wide<0, false, |", "padded SELL-64, one workgroup per slice"),
    "jag-pw": ("k_sell_pw<0, false, |", "jagged SELL-64, wave-product-parallel"),
    "padded+vt16": ("k_sell_vt<0, false, |, false>(hve::SpArgs)", "padded SELL-64 with a 16-bit value table"),
    "jagged+vt16": ("k_sell_vt<0, false, |, true>(hve::SpArgs)", "jagged SELL-64 with a 16-bit value table"),
}


def committed_traffic(n, kname):
    """HBM bytes per launch of the finest residual SpMV from the newest
    committed rocprofv3 PMC summary for this workload (scripts/pmc_traffic.py),
    or None when that summary measured another kernel / layout (every kernel
    name it matched must contain both halves of kname around the batch width).
    Counters need their own profiler passes, so the bench reports the committed
    measurement of the same kernel and grid."""
    found = []
    for dirpath, _, files in os.walk(PROFILE_DIR):
        if f"pmc_traffic_{n}.json" in files:
            found.append(os.path.join(dirpath, f"pmc_traffic_{n}.json"))
    if not found:
        return None
    best = sorted(found)[-1]  # profiles/rNN/<seq>_<name>/: the newest measurement
    with open(best) as f:
        d = json.load(f)
    names = d.get("kernel_names", [])
    pre, post = kname.split("|")
    if not names or not all(pre in nm and post in nm[nm.index(pre) + len(pre):] for nm in names if pre in nm) \
            or not all(pre in nm for nm in names):
        return None
    return round(d["traffic_bytes"], 0)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class heartbeat:
    """Prints a progress line every `every` s while a long host phase (the
    setup at 512^3 takes minutes) runs inside a ctypes call (GIL released)."""

    def __init__(self, what, every=30.0):
        import threading
        self.what, self.every, self.t0 = what, every, time.time()
        self.stop = threading.Event()
        self.th = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        while not self.stop.wait(self.every):
            log(f"[bench] {self.what}: {time.time() - self.t0:.0f}s")

    def __enter__(self):
        self.th.start()
        return self

    def __exit__(self, *exc):
        self.stop.set()


def slab_rows(nx, ny, nz, world):
    """[(first_row, rows)] of each rank's z-slab when GenerateLaplacian[27pt]
    splits nx x ny x nz over a 1 x 1 x world process grid: the planes by
    hypre_GeneratePartitioning (seq_mv/genpart.c:18: the first nz % world
    slabs one plane more), each slab's rows in natural order after the
    previous slab's (par_laplace.c:363 hypre_map with P = Q = 1)."""
    size, rest = divmod(nz, world)
    out, z0 = [], 0
    for r in range(world):
        nzl = size + (1 if r < rest else 0)
        out.append((z0 * nx * ny, nzl * nx * ny))
        z0 += nzl
    return out


def sha256_f64(v):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(v, dtype="<f8").tobytes()).hexdigest()


def slab_digests_of(x, nx, ny, nz, worlds=(2, 4, 8)):
    """sha256 of the whole iterate and of its z-slabs as an N-rank run would
    own them, for each N in worlds."""
    out = {"1": [sha256_f64(x)]}
    for w in worlds:
        if w <= nz:
            out[str(w)] = [sha256_f64(x[f:f + c]) for f, c in slab_rows(nx, ny, nz, w)]
    return out


def slab_starts(nx, ny, nz, world):
    """Level-0 row starts of the world-rank z-slab run (slab_rows)."""
    cuts = slab_rows(nx, ny, nz, world)
    return [f for f, _ in cuts] + [nx * ny * nz]


GOLDEN_DIGESTS = os.path.join(ROOT, "tests", "golden", "slab_digests.json")
# Workloads no single process can hold, so no one-GPU reference exists (the
# N-rank line then reports "equal": null with this reason)
NO_REFERENCE = {
    "512x512x512 stencil27": (
        "no one-process reference exists: GenerateLaplacian27pt at 512^3 has 3.62e9 nonzeros, past the 2^31 - 1 "
        "entries a 32-bit CSR row pointer addresses (the reference's default 32-bit HYPRE_Int build has the same "
        "bound for one process); the 8-rank run holds 4.5e8 a rank.  The same code is pinned at 256^3 "
        "(tests/golden/slab_digests.json, 256x256x256 stencil27, columns 2 / 4 / 8)"),
}


def digest_key(args, nx, ny, nz, iters):
    """The workload a slab digest belongs to: grid, operator, method, the
    parity iterations from x = 0 with rhs = ones."""
    return (f"{nx}x{ny}x{nz} stencil{args.stencil} coef{args.coef} agg{args.agg} relax{args.relax} "
            f"coarsen{args.coarsen} solver{args.solver} iters{iters}")


def golden_slab_digests(key):
    """The committed digests of workload `key` (tests/golden/slab_digests.json,
    merged by scripts/golden_digests.py from one-GPU lines whose iterate was
    bitwise equal to the C oracle's): column "1" the whole iterate of the
    one-process setup, column "N" the slabs of the N-rank setup's iterate (a
    one-GPU run under the rank emulation of N z-slab ranks, bench.py
    --emulate N: hypre's N-process rules, the contract of every N-rank run),
    or None."""
    try:
        with open(GOLDEN_DIGESTS) as f:
            return json.load(f).get(key)
    except (OSError, ValueError):
        return None


def oracle_cpu_baseline(amg, nrows, n, pcg, args):
    """The reference's CPU solve path, restated in C (oracle/oracle.c, the
    parity checker) and run with OpenMP over rows on this host's cores, on the
    hierarchy `amg` (one-process setup) with rhs = ones, from x = 0, for
    args.parity_iters iterations (the sample; about 10 s at 512^3 on 16
    threads).  Returns (cpu_baseline dict, the oracle's iterate, iterations):
    the bench then runs the GPU for the same iterations from the same start
    and compares the iterates bit for bit."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py

    O = oracle_py.OracleAMG(amg)
    bh = np.ones(nrows)
    u = np.zeros(nrows)

    def cpu_run(k):
        u[:] = 0.0
        if pcg:
            return O.pcg(bh, u, 0.0, k, 1)[0]
        return O.solve(bh, u, 1e-300, k)["iterations"]

    iters = args.parity_iters
    tc = time.perf_counter()
    done = cpu_run(iters)
    tcpu = time.perf_counter() - tc
    threads = oracle_py.num_threads()
    what = "PCG iterations (one V-cycle preconditioner each)" if pcg else "solve iterations (V-cycle + residual norm)"
    cpu = {"value": round(nrows * done / tcpu, 1), "unit": "DOF/s", "cores": threads, "kind": "port",
           "sample": f"{done} {what} of the same {n} hierarchy by the C oracle (oracle/oracle.c), "
                     f"OpenMP {threads} threads, {tcpu:.1f}s"}
    log(f"[bench] cpu oracle: {cpu['value']:.3e} DOF/s ({done} iterations, {tcpu:.1f}s, {threads} threads)")
    return cpu, u, done, O


def gpu_parity(hv, amg, krylov, A, b, x, u_oracle, iters, pcg):
    """The GPU solve from x = 0 for the oracle's iterations, compared with the
    oracle's iterate: every row sum keeps the reference's order, so a V-cycle
    solve must agree bit for bit (PCG's dot products reduce in another order:
    its iterate is compared at a stated tolerance instead)."""
    x.fill(0.0)
    if pcg:
        krylov.set(max_iter=iters)
        krylov.solve(A, b, x)
    else:
        amg.set(max_iter=iters)
        amg.solve(A, b, x)
    xg = x.get()
    if not pcg:
        same = bool(np.array_equal(xg, u_oracle))
        diff = 0.0 if same else float(np.max(np.abs(xg - u_oracle)))
        res = {"kind": "bitwise", "equal": same, "iterations": iters, "rows": int(xg.size),
               "max_abs_diff": diff}
        tag = "bitwise" if same else "MISMATCH"
    else:
        rel = float(np.linalg.norm(xg - u_oracle) / max(np.linalg.norm(u_oracle), 1e-300))
        ok = rel <= 1e-9
        res = {"kind": "rtol 1e-9 (PCG reductions reorder)", "equal": ok, "iterations": iters,
               "rows": int(xg.size), "rel_diff": rel}
        tag = "rtol1e-9" if ok else "MISMATCH"
    log(f"[bench] parity: GPU vs oracle after {iters} iterations from x = 0 on {xg.size} rows: {tag}")
    return tag, res


def pcg_parity(hv, amg, A, b, x, O, nrows, iters):
    """configs[2]'s solver on the bench's hierarchy: BoomerAMG-PCG (ij
    -solver 1: two-norm PCG, krylov/pcg.c:271, one V-cycle per iteration from
    a cleared z) for `iters` iterations from x = 0 on the GPU and in the C
    oracle.  PCG's dot products reduce in another order than the oracle's, so
    the iterate is compared at rtol 1e-9 with equal iteration counts, as the
    PCG tests do (tests/test_gpu_parity.py)."""
    amg.set(tol=0.0, max_iter=1)  # the preconditioner: one cycle (ij.c -solver 1)
    kr = hv.PCG(tol=0.0, max_iter=iters, two_norm=1)
    kr.set_precond_amg(amg, setup=False)  # the hierarchy is set up already
    kr.setup(A, b, x)
    x.fill(0.0)
    it_g, rr_g = kr.solve(A, b, x)
    xg = x.get()
    kr.destroy()
    u = np.zeros(nrows)
    it_o, rr_o = O.pcg(np.ones(nrows), u, 0.0, iters, 1)
    rel = float(np.linalg.norm(xg - u) / max(np.linalg.norm(u), 1e-300))
    ok = rel <= 1e-9 and it_g == it_o == iters
    log(f"[bench] parity_pcg: {iters} PCG iterations on {nrows} rows: GPU vs oracle rel. diff {rel:.3e}, "
        f"final rel. residual {rr_g:.6e} vs {rr_o:.6e}: {'rtol1e-9' if ok else 'MISMATCH'}")
    return {"kind": "rtol 1e-9 (PCG reductions reorder)", "equal": ok, "iterations": int(it_g),
            "oracle_iterations": int(it_o), "rows": int(nrows), "rel_diff": rel,
            "final_rel_res": rr_g, "oracle_final_rel_res": rr_o}


def tol_key(tol):
    """JSON key of the time-to-solution entry: iters_to_1e-8 for 1e-8."""
    return "iters_to_" + f"{tol:g}".replace("e-0", "e-")


def iters_to_tol(hv, amg, A, b, x, n, tol=1e-8, oracle=None):
    """Time to solution, the number a hypre user sees: BoomerAMG as the solver
    (ij -solver 0) and as PCG's preconditioner (ij -solver 1, one V-cycle an
    iteration) from x = 0 with rhs = ones, each to the relative residual tol,
    on the GPU; oracle (an OracleAMG of the same hierarchy): the C oracle's
    counts beside them."""
    out = {"tol": tol}
    amg.set(tol=tol, max_iter=1000, min_iter=0)
    x.fill(0.0)
    t0 = time.perf_counter()
    it, rr = amg.solve(A, b, x)
    out["vcycle"] = {"iterations": int(it), "rel_res": rr, "seconds": round(time.perf_counter() - t0, 3)}
    amg.set(tol=0.0, max_iter=1)  # the preconditioner: one cycle
    kr = hv.PCG(tol=tol, max_iter=1000, two_norm=1)
    kr.set_precond_amg(amg, setup=False)
    kr.setup(A, b, x)
    x.fill(0.0)
    t0 = time.perf_counter()
    it, rr = kr.solve(A, b, x)
    out["pcg"] = {"iterations": int(it), "rel_res": rr, "seconds": round(time.perf_counter() - t0, 3)}
    kr.destroy()
    if oracle is not None:
        u = np.zeros(n)
        st = oracle.solve(np.ones(n), u, tol, 1000)
        out["vcycle"]["oracle_iterations"] = st["iterations"]
        u[:] = 0.0
        ito, _ = oracle.pcg(np.ones(n), u, tol, 1000, 1)
        out["pcg"]["oracle_iterations"] = int(ito)
    log(f"[bench] iterations to {tol:g}: V-cycle {out['vcycle']['iterations']}"
        f"{' (oracle ' + str(out['vcycle'].get('oracle_iterations')) + ')' if oracle is not None else ''}, "
        f"PCG {out['pcg']['iterations']}"
        f"{' (oracle ' + str(out['pcg'].get('oracle_iterations')) + ')' if oracle is not None else ''}")
    return out


def hierarchy_digest(amg):
    """sha256 over every level's A, P, R (row pointers, columns, value bits),
    CF marker and l1 norms: one level at a time, so two 256^3 hierarchies can
    be compared without holding both."""
    import hashlib
    h = hashlib.sha256()
    nl = amg.num_levels()
    for l in range(nl):
        for w in (0, 1, 2):
            if w and l == nl - 1:
                continue
            ip, jj, vv, shp = amg.level_matrix(l, w)
            h.update(np.asarray(shp, dtype=np.int64).tobytes())
            for arr in (ip, jj, vv):
                h.update(np.ascontiguousarray(arr).tobytes())
        for w in (0, 1):
            h.update(np.ascontiguousarray(amg.level_vector(l, w)).tobytes())
    return h.hexdigest()


def setup_parity(hv, args, n):
    """The device setup (Setup's default: ext+i, truncation, R = P^T and RAP
    on the GPU) against the host setup (SetupHost, the restatement pinned to
    the reference's saved runs) at n^3: every level's bytes must agree."""
    cx, cy, cz = (float(v) for v in args.coef.split(","))
    digests = []
    t0 = time.time()
    for host in (False, True):
        A = (hv.ParCSRMatrix.laplacian27(n, n, n) if args.stencil == 27
             else hv.ParCSRMatrix.laplacian(n, n, n, cx=cx, cy=cy, cz=cz))
        amg = hv.BoomerAMG(**amg_settings(hv, False, args.agg, args.relax, args.coarsen))
        if host:
            amg.setup_host(A)
        else:
            amg.setup(A)
        digests.append((hierarchy_digest(amg), amg.num_levels()))
        amg.destroy()
        A.destroy()
    ok = digests[0] == digests[1]
    log(f"[bench] setup parity at {n}^3: device setup {'==' if ok else '!='} host setup "
        f"({digests[0][1]} levels, {time.time() - t0:.1f}s)")
    return {"kind": "sha256 of every level's A, P, R, CF and l1 bytes", "size": f"{n}^3", "equal": ok,
            "levels": digests[0][1], "device_digest": digests[0][0], "host_digest": digests[1][0]}


def amg_settings(hv, pcg, agg=0, relax=18, coarsen=8):
    """The bench's BoomerAMG: PMIS, ext+i (Pmx 4), l1-Jacobi down/up,
    Gaussian elimination on the coarsest level (ij -pmis -rlx 18); agg > 0:
    that many aggressive levels with multipass interpolation (configs[4],
    ij -agg_nl).  relax < 0 keeps BoomerAMG's default smoothers (l1 hybrid
    Gauss-Seidel 13 down / 14 up, automatic block count); coarsen 10 = HMIS."""
    kw = hv.ij_amg_defaults(1 if pcg else 0)
    kw.update(coarsen_type=coarsen, interp_type=6, P_max_elmts=4, agg_num_levels=agg)
    if relax >= 0:
        kw.update(relax_type=relax)
    return kw


def smoother_name(relax):
    if relax < 0:
        return "l1 hybrid Gauss-Seidel (relax 13 down / 14 up, BoomerAMG's default)"
    if relax == 18:
        return "l1-Jacobi (relax 18) down/up"
    return f"relax {relax} down/up"


def global_grid(args, world):
    """(nx, ny, nz) of the global problem.  Strong (the default): --grid, or
    n^3, split over the ranks in z-slabs (ij -n is the global size, ij.c:1780;
    hypre_GeneratePartitioning gives the first nz % N slabs one plane more).
    --weak: n x n x (n N), n^3 rows per rank."""
    if args.grid:
        nx, ny, nz = (int(v) for v in args.grid.split(","))
    else:
        nx = ny = nz = args.n
    if args.weak:
        nz *= world
    return nx, ny, nz


def peak_rss_gb():
    import resource
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6


def run_rank(hv, args, comm, rank, world, barrier, max_over_ranks, gather, n=None, light=False):
    """One rank's part of the bench; returns the JSON dict on rank 0.  light:
    a secondary size (no CPU baseline, no stream calibration)."""
    import torch

    t0 = time.time()
    cx, cy, cz = (float(v) for v in args.coef.split(","))
    if n is None:
        nx, ny, nz = global_grid(args, world)
    else:
        nx = ny = nz = n

    def gen(**part):
        if args.stencil == 27:
            return hv.ParCSRMatrix.laplacian27(nx, ny, nz, **part)
        return hv.ParCSRMatrix.laplacian(nx, ny, nz, cx=cx, cy=cy, cz=cz, **part)

    if comm is not None:
        # rank r owns z-slab r of the P x Q x R = 1 x 1 x world process grid
        A = gen(comm=comm, P=1, Q=1, R=world, p=0, q=0, r=rank)
    else:
        A = gen()
    nrows = A.n
    gn = nx * ny * nz
    pcg = args.solver == "pcg"
    first = A.first if comm is not None else 0
    b = hv.ParVector(nrows, np.ones(nrows), comm=comm, first=first, global_n=gn)
    x = hv.ParVector(nrows, np.zeros(nrows), comm=comm, first=first, global_n=gn)
    krylov = None
    if pcg:
        # ij -solver 1: PCG (two-norm) preconditioned by one BoomerAMG V-cycle
        amg = hv.BoomerAMG(**amg_settings(hv, True, args.agg, args.relax, args.coarsen))
        krylov = hv.PCG(tol=0.0, max_iter=max(1, args.warmup), two_norm=1)
        krylov.set_precond_amg(amg)
        with heartbeat(f"rank {rank} setup"):
            krylov.setup(A, b, x)
    else:
        kw = amg_settings(hv, False, args.agg, args.relax, args.coarsen)
        kw.update(tol=1e-300, max_iter=args.warmup, min_iter=0)
        amg = hv.BoomerAMG(**kw)
        with heartbeat(f"rank {rank} setup"):
            amg.setup(A)
    t_setup = time.time() - t0
    rss_setup = peak_rss_gb()
    g, o, c = amg.complexities()
    if rank == 0:
        log(f"[bench] ranks={world} grid={nx}x{ny}x{nz} rows/rank={nrows} levels={amg.num_levels()} grid={g:.4f} "
            f"op={o:.4f} setup={t_setup:.1f}s peak RSS {rss_setup:.1f} GB")
    # warmup (also instantiates the cycle hipGraph)
    if args.warmup > 0:
        if pcg:
            krylov.set(max_iter=args.warmup)
            krylov.solve(A, b, x)
        else:
            amg.set(max_iter=args.warmup)
            amg.solve(A, b, x)
    x.fill(0.0)
    if pcg:
        krylov.set(max_iter=args.steps)
    else:
        amg.set(max_iter=args.steps)
    torch.cuda.synchronize()
    barrier()
    t_start = time.perf_counter()
    it, rr = (krylov if pcg else amg).solve(A, b, x)
    torch.cuda.synchronize()
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t_start)
    assert it == args.steps, (it, args.steps)
    ms_per_step = elapsed / args.steps * 1e3
    value = gn * args.steps / elapsed
    if rank == 0:
        log(f"[bench] {args.steps} steps in {elapsed*1e3:.2f} ms -> {ms_per_step:.3f} ms/step, rel.res {rr:.3e}")

    # roofline: finest-level SpMV (the dominant kernel), HIP events on the solver stream.
    # achieved = the bytes its stored layout must move per launch / launch time
    # (hypreve_BenchFineSpMVStoredBytes); the CSR-equivalent rate (12 B a
    # nonzero) is reported beside it.
    spmv_ms, csr_bytes = amg.bench_fine_spmv(args.spmv_reps)
    stored_bytes = amg.fine_spmv_stored_bytes()
    achieved = stored_bytes / (spmv_ms * 1e-3) / 1e9
    csr_gbs = csr_bytes / (spmv_ms * 1e-3) / 1e9
    aniso = args.coef != "1,1,1"
    default_op = args.stencil == 7 and not aniso and not args.agg and args.relax == 18 and args.coarsen == 8
    layout0 = amg.level_layout(0, 0)
    kname, kdesc = KERNEL_OF_LAYOUT[layout0]
    # the committed PMC summary (scripts/pmc_traffic.py) measured the default
    # operator's finest residual kernel at this size; reported only for the same kernel
    traffic = committed_traffic(nx, kname) if (default_op and world == 1 and nx == ny == nz) else None
    # every large operator of the cycle, each timed alone with HIP events (bytes
    # of its stored layout + vectors per launch)
    per_kernel = []
    nl = amg.num_levels()
    for lvl, which, what in ((0, 0, "A0 residual"), (0, 1, "P0 prolongation"), (0, 2, "R0 restriction"),
                             (1, 0, "A1 residual"), (1, 1, "P1 prolongation"), (1, 2, "R1 restriction"),
                             (2, 0, "A2 residual")):
        if lvl >= nl or (which and lvl >= nl - 1):
            continue
        ms_k, csr_k, _ = amg.bench_level_op(lvl, which, max(5, args.spmv_reps // 2))
        sb_k = amg.level_op_stored_bytes(lvl, which)
        per_kernel.append({"op": what, "layout": amg.level_layout(lvl, which), "avg_ms": round(ms_k, 4),
                           "stored_bytes": round(sb_k), "csr_bytes": round(csr_k),
                           "gbs": round(sb_k / (ms_k * 1e-3) / 1e9, 1),
                           "frac": round(sb_k / (ms_k * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)})
        if rank == 0:
            log(f"[bench] {what:16s} {per_kernel[-1]['layout']:12s} {ms_k:.4f} ms  "
                f"{sb_k / 1e9:.3f} GB stored -> {per_kernel[-1]['gbs']:.0f} GB/s ({per_kernel[-1]['frac']:.3f})")
    # the box's achievable read bandwidth: a grid-stride 8 B/lane stream over 2 GiB
    stream_n = (1 << 31) // 8
    stream_gbs = stream_n * 8 / (hv.bench_stream(8, stream_n, 3 if light else 10) * 1e-3) / 1e9
    # and its read/write mix: 5 double streams read and one written per element
    mix_n = (1 << 27)
    mix_gbs = mix_n * 48 / (hv.bench_stream(-5, mix_n, 3 if light else 10) * 1e-3) / 1e9
    if args.calib:
        for eb in (2, 4, 8):
            hv.bench_stream(eb, (1 << 29) // eb, 1)
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "kernel": f"{kname.replace('|', 'NW' if layout0 == 'grid-stencil' else 'B').split('(')[0]} finest level (r = b - A x), {kdesc}",
            "layout": layout0,
            "avg_ms": round(spmv_ms, 4), "bytes_per_launch": stored_bytes,
            "csr_bytes_per_launch": csr_bytes, "csr_equivalent_gbs": round(csr_gbs, 1),
            "stream_read_gbs": round(stream_gbs, 1), "frac_of_stream": round(achieved / stream_gbs, 4),
            "stream_mix_gbs": round(mix_gbs, 1), "frac_of_mix_stream": round(achieved / mix_gbs, 4),
            "per_kernel": per_kernel}
    if world == 1 and comm is None and not light:
        # the same finest residual through the general per-entry path: the
        # operator uploaded alone in padded SELL-64 (32-bit column + f64 value
        # per stored entry, what any variable-coefficient operator streams),
        # same traversal, HIP events
        g_ms, g_bytes, _ = A.bench_operator(op=0, policy=1, nbands=8, reps=max(5, args.spmv_reps // 2))
        roof["general"] = {"layout": "padded SELL-64, 32-bit column + f64 value per entry (policy 1)",
                           "avg_ms": round(g_ms, 4), "bytes_per_launch": round(g_bytes),
                           "achieved": round(g_bytes / (g_ms * 1e-3) / 1e9, 1),
                           "frac": round(g_bytes / (g_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
        if rank == 0:
            log(f"[bench] general path (padded, f64 values): {g_ms:.4f} ms, {g_bytes / 1e9:.3f} GB -> "
                f"{roof['general']['achieved']:.0f} GB/s ({roof['general']['frac']:.3f})")
    if rank == 0:
        log(f"[bench] read stream {stream_gbs:.0f} GB/s, 5:1 read/write mix {mix_gbs:.0f} GB/s; "
            f"fine SpMV at {achieved / stream_gbs:.3f} / {achieved / mix_gbs:.3f} of them")
        log(f"[bench] fine SpMV {spmv_ms:.4f} ms, {stored_bytes/1e9:.3f} GB stored -> {achieved:.1f} GB/s "
            f"(CSR-equivalent {csr_gbs:.1f} GB/s); host peak RSS {peak_rss_gb():.1f} GB")

    cpu, parity, parity_detail, parity_pcg, slab, to_tol = None, None, None, None, None, None
    if world == 1 and comm is None and args.iters_tol > 0 and not pcg:
        O_tol = None
        if light and args.cpu_cycles > 0:  # the secondary size: the C oracle's counts beside the GPU's
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle_py
            O_tol = oracle_py.OracleAMG(amg)
        to_tol = iters_to_tol(hv, amg, A, b, x, nrows, args.iters_tol, O_tol)
        del O_tol
        amg.set(tol=1e-300, min_iter=0)
    if rank == 0 and not light and args.cpu_cycles > 0 and world == 1 and comm is None:
        cpu, u_orc, iters, O = oracle_cpu_baseline(amg, nrows, f"{nx}x{ny}x{nz}", pcg, args)
        parity, parity_detail = gpu_parity(hv, amg, krylov, A, b, x, u_orc, iters, pcg)
        if not pcg:
            # the oracle-equal iterate of the one-process setup (the N-rank
            # references come from --emulate N lines)
            key = digest_key(args, nx, ny, nz, iters)
            slab = {"iterations": iters, "key": key, "equal_to_oracle": parity_detail["equal"],
                    "digests": {"1": [sha256_f64(u_orc)]}}
            log(f"[bench] slab digests ({key}): whole {slab['digests']['1'][0][:16]}...")
        del u_orc
        if not pcg and args.pcg_iters > 0:
            parity_pcg = pcg_parity(hv, amg, A, b, x, O, nrows, args.pcg_iters)
        del O
    if not light and world > 1 and args.parity_iters > 0 and not pcg:
        # bench contract: the CPU baseline is timed at N = 1 only.  An N-rank
        # run follows hypre's N-process setup rules, which one GPU reproduces
        # under the rank emulation (bench.py --emulate N: the same iterate bit
        # for bit, checked there against the C oracle); here every rank solves
        # the same iterations from x = 0 and rank 0 compares the gathered
        # 32-byte digests of the rank iterates with that reference's slabs
        # (the halo exchange of par_csr_communication.c:298 is on this path)
        x.fill(0.0)
        amg.set(max_iter=args.parity_iters)
        amg.solve(A, b, x)
        mine = (A.first, sha256_f64(x.get()))
        got = sorted(gather(mine))
        if rank == 0:
            key = digest_key(args, nx, ny, nz, args.parity_iters)
            ref = golden_slab_digests(key)
            cuts = slab_rows(nx, ny, nz, world)
            dig = [d for _, d in got]
            same_cut = [f for f, _ in got] == [f for f, _ in cuts]
            want = (ref or {}).get(str(world))
            equal = (dig == want and same_cut) if want is not None else None
            parity = {"kind": f"slab sha256 vs the one-GPU rank emulation of {world} ranks", "equal": equal,
                      "iterations": args.parity_iters, "key": key, "rank_digests": dig,
                      "rank_first_rows": [f for f, _ in got],
                      "reference": (f"tests/golden/slab_digests.json column {world} (bench.py --emulate {world} "
                                    "line: one GPU, hypreve_BoomerAMGSetRankEmulation, its iterate bitwise equal "
                                    "to the C oracle's on that hierarchy)") if want is not None else
                      NO_REFERENCE.get(key.split()[0] + " " + key.split()[1],
                                       f"no committed {world}-rank digests for this workload: run bench.py "
                                       f"--emulate {world} on one GPU and compare rank_digests with its digests")}
            log(f"[bench] slab parity vs the {world}-rank emulation after {args.parity_iters} iterations: "
                f"{'bitwise' if equal else ('MISMATCH' if equal is False else 'no reference')}")
    comm_stats = None
    if world > 1:
        # this rank's communication per V-cycle, per level (the solve loop adds
        # one level-0 exchange for its residual and one all-reduce for its norm)
        cc = amg.cycle_comm_stats()
        comm_stats = {"exchanges": sum(c["exchanges"] for c in cc), "bytes": sum(c["bytes"] for c in cc),
                      "allgathers": sum(c["allgathers"] for c in cc),
                      "allgather_bytes": sum(c["allgather_bytes"] for c in cc),
                      "allreduces": sum(c["allreduces"] for c in cc),
                      "per_level": [[c["exchanges"], c["bytes"]] for c in cc]}
    stats = gather({"rank": rank, "rows": nrows, "setup_s": round(t_setup, 1), "setup_peak_rss_gb": round(rss_setup, 1),
                    "peak_rss_gb": round(peak_rss_gb(), 1), "omp_threads": int(os.environ.get("OMP_NUM_THREADS", "0")),
                    "cycle_comm": comm_stats})
    nlev = amg.num_levels()
    for obj in ((krylov,) if pcg else ()) + (amg, A, b, x):
        obj.destroy()  # release host and device memory before a secondary size runs
    if rank != 0:
        return None
    strong = not args.weak
    split = f"{world} z-slab row blocks" if world > 1 else "one row block"
    scaled = "global problem, fixed as N grows" if strong else f"{nx}x{ny}x{nz // world} per GPU"
    opname = f"{'anisotropic diffusion (' + args.coef + ')' if aniso else 'Laplacian'}"
    out = {
        "metric": "BoomerAMG V-cycle DOF/s + finest-level SpMV GB/s vs HBM peak, 1/2/4/8 GPU",
        "value": round(value, 1),
        "unit": "DOF/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": f"synthetic ({'GenerateLaplacian27pt' if args.stencil == 27 else 'GenerateLaplacian 7-point'}"
                f"{'' if default_op else ', coefficients ' + args.coef}, rhs = ones)",
        "config": {"workload": f"3D {args.stencil}-point {opname} {nx}x{ny}x{nz} ({scaled}; {split})"
                               f", {'BoomerAMG-PCG (one V-cycle per PCG iteration)' if pcg else 'BoomerAMG V-cycle'}"
                               f", {'HMIS' if args.coarsen == 10 else 'PMIS'} + ext+i (Pmx 4)"
                               f"{f', {args.agg} aggressive level(s) (multipass)' if args.agg else ''}"
                               f", {smoother_name(args.relax)}, Gaussian elimination coarsest",
                   "global_rows": gn, "rows_per_gpu": nrows, "levels": nlev, "grid_complexity": round(g, 6),
                   "operator_complexity": round(o, 6), "setup_s": round(t_setup, 1),
                   "per_rank": stats,
                   "parallelism": f"rows{world}, {'strong' if strong else 'weak'}"},
        "roofline": roof,
        "cpu_baseline": cpu,
        "parity": parity,
    }
    if parity_detail is not None:
        out["parity_detail"] = parity_detail
    if to_tol is not None:
        out[tol_key(args.iters_tol)] = to_tol
    if parity_pcg is not None:
        out["parity_pcg"] = parity_pcg
    if slab is not None:
        out["slab_digests"] = slab
    if world > 1:
        out["cpu_baseline_note"] = ("timed at N = 1 only (bench contract); strong scaling: the N = 1 line runs "
                                    "the same global problem") if strong else "timed at N = 1 only (bench contract)"
    return out


def gs_leg(hv, args, n):
    """BoomerAMG's default smoothers (l1 hybrid Gauss-Seidel 13 down / 14 up,
    par_relax.c:4340 / :4732, automatic blocks) on the n^3 7-point Laplacian,
    the bench's other settings unchanged: args.steps solve iterations timed as
    the headline is, then args.parity_iters iterations from x = 0 compared
    bit for bit with the C oracle on the same hierarchy."""
    import torch

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py

    t0 = time.time()
    A = hv.ParCSRMatrix.laplacian(n, n, n)
    kw = amg_settings(hv, False, 0, -1, args.coarsen)
    kw.update(tol=1e-300, max_iter=args.warmup, min_iter=0)
    amg = hv.BoomerAMG(**kw)
    with heartbeat("hybrid GS setup"):
        amg.setup(A)
    t_setup = time.time() - t0
    b = hv.ParVector(A.n, np.ones(A.n))
    x = hv.ParVector(A.n, np.zeros(A.n))
    if args.warmup > 0:
        amg.solve(A, b, x)
    x.fill(0.0)
    amg.set(max_iter=args.steps)
    torch.cuda.synchronize()
    ts = time.perf_counter()
    it, rr = amg.solve(A, b, x)
    torch.cuda.synchronize()
    el = time.perf_counter() - ts
    assert it == args.steps, (it, args.steps)
    iters = args.parity_iters
    x.fill(0.0)
    amg.set(max_iter=iters)
    amg.solve(A, b, x)
    xg = x.get()
    O = oracle_py.OracleAMG(amg)
    u = np.zeros(A.n)
    O.solve(np.ones(A.n), u, 1e-300, iters)
    same = bool(np.array_equal(xg, u))
    out = {"config": f"3D 7-point Laplacian {n}^3, BoomerAMG V-cycle, PMIS + ext+i (Pmx 4), l1 hybrid Gauss-Seidel "
                     f"13 down / 14 up (BoomerAMG's default smoothers, automatic blocks), Gaussian elimination coarsest",
           "value": round(A.n * args.steps / el, 1), "unit": "DOF/s", "ms_per_step": round(el / args.steps * 1e3, 4),
           "steps": args.steps, "levels": amg.num_levels(), "setup_s": round(t_setup, 1),
           "parity": {"kind": "bitwise", "equal": same, "iterations": iters, "rows": A.n}}
    log(f"[bench] hybrid GS {n}^3: {out['ms_per_step']:.3f} ms/step, setup {t_setup:.1f}s, parity vs oracle after "
        f"{iters} iterations: {'bitwise' if same else 'MISMATCH'}")
    for o in (amg, A, b, x):
        o.destroy()
    return out


def emulated_reference(hv, args, world):
    """The reference of a world-rank line, made on one GPU: the global problem
    set up under the rank emulation of world z-slab ranks
    (hypreve_BoomerAMGSetRankEmulation: hypre's N-process setup rules, which
    every N-rank setup of the library follows), solved args.parity_iters
    iterations from x = 0, and checked bit for bit against the C oracle run on
    the same hierarchy.  Prints one JSON line whose slab_digests (column
    `world`: the iterate cut at the ranks' slabs) scripts/golden_digests.py
    merges into tests/golden/slab_digests.json."""
    import torch

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py

    torch.cuda.set_device(0)
    hv.init()
    cx, cy, cz = (float(v) for v in args.coef.split(","))
    nx, ny, nz = global_grid(args, 1)
    if world > nz:
        raise SystemExit(f"--emulate {world}: fewer planes ({nz}) than ranks")
    t0 = time.time()
    A = (hv.ParCSRMatrix.laplacian27(nx, ny, nz) if args.stencil == 27
         else hv.ParCSRMatrix.laplacian(nx, ny, nz, cx=cx, cy=cy, cz=cz))
    n = A.n
    iters = args.parity_iters
    kw = amg_settings(hv, False, args.agg, args.relax, args.coarsen)
    kw.update(tol=1e-300, max_iter=iters, min_iter=0)
    amg = hv.BoomerAMG(**kw)
    amg.set_rank_emulation(slab_starts(nx, ny, nz, world))
    with heartbeat(f"setup under the {world}-rank emulation"):
        amg.setup(A)
    t_setup = time.time() - t0
    b = hv.ParVector(n, np.ones(n))
    x = hv.ParVector(n, np.zeros(n))
    it, rr = amg.solve(A, b, x)
    xg = x.get()
    with heartbeat("oracle"):
        O = oracle_py.OracleAMG(amg)
        u = np.zeros(n)
        st = O.solve(np.ones(n), u, 1e-300, iters)
    same = bool(np.array_equal(xg, u)) and st["iterations"] == it == iters
    key = digest_key(args, nx, ny, nz, iters)
    dig = {str(world): [sha256_f64(u[f:f + c]) for f, c in slab_rows(nx, ny, nz, world)]}
    g, o, c = amg.complexities()
    log(f"[bench] --emulate {world}: {nx}x{ny}x{nz}, {amg.num_levels()} levels, setup {t_setup:.1f}s, "
        f"GPU vs oracle after {iters} iterations: {'bitwise' if same else 'MISMATCH'}")
    out = {"kind": f"one-GPU reference of the {world}-rank run (rank emulation)", "n_gpus": 1,
           "emulated_ranks": world, "setup_path": amg.setup_path(), "levels": amg.num_levels(),
           "grid_complexity": round(g, 6), "operator_complexity": round(o, 6), "setup_s": round(t_setup, 1),
           "rel_res": rr, "slab_digests": {"iterations": iters, "key": key, "equal_to_oracle": same, "digests": dig}}
    print(json.dumps(out), flush=True)
    return 0 if same else 1


def visible_gpus():
    """GPUs this process may use, counted without loading the HIP runtime: the
    KFD topology nodes with SIMDs (the GPUs; CPU nodes have none), limited by
    a *_VISIBLE_DEVICES list when the launcher set one.  The launcher parent
    then starts torch.distributed.run with nothing of the GPU initialised."""
    topo = "/sys/class/kfd/kfd/topology/nodes"
    n = 0
    try:
        for node in os.listdir(topo):
            try:
                with open(os.path.join(topo, node, "properties")) as f:
                    props = dict(ln.split()[:2] for ln in f if len(ln.split()) >= 2)
                if int(props.get("simd_count", "0")) > 0:
                    n += 1
            except (OSError, ValueError):
                continue
    except OSError:
        return 0
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([t for t in v.split(",") if t.strip()]))
    return n


def rank_threads():
    """OpenMP threads of this rank's host setup: the host cores this process may
    use, shared by the ranks of the node (LOCAL_WORLD_SIZE), and no more than an
    OMP_NUM_THREADS the launcher set.  Set before the OpenMP runtime loads."""
    lw = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
    share = len(os.sched_getaffinity(0))
    per = max(1, share // max(1, lw))
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        per = min(per, int(env))
    os.environ["OMP_NUM_THREADS"] = str(per)
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=512,
                    help="grid edge of the global n^3 problem (512: configs[2]-[4]'s 512^3, the north-star size), "
                         "split over the ranks in z-slabs; with --weak n^3 rows per GPU")
    ap.add_argument("--grid", default="",
                    help="nx,ny,nz of the global grid instead of n^3 (e.g. 512,512,64: one rank's share of the "
                         "8-GPU 512^3 problem, for a one-GPU rehearsal)")
    ap.add_argument("--weak", action="store_true",
                    help="weak scaling: n^3 rows per GPU (n x n x n*N global) instead of the global n^3")
    ap.add_argument("--secondary-n", type=int, default=256,
                    help="one GPU: also measure this size (configs[1]'s 256^3) into 'secondary' (0 = skip)")
    ap.add_argument("--stencil", type=int, choices=[7, 27], default=7,
                    help="7: GenerateLaplacian (configs[1], the bench line); 27: GenerateLaplacian27pt (configs[3])")
    ap.add_argument("--coef", default="1,1,1",
                    help="cx,cy,cz of the 7-point operator; e.g. 0.001,1,1 for configs[4]'s anisotropic diffusion")
    ap.add_argument("--agg", type=int, default=0,
                    help="aggressive coarsening levels (configs[4]: with --coef 0.001,1,1), multipass interpolation")
    ap.add_argument("--relax", type=int, default=18,
                    help="relax type down/up (18: l1-Jacobi, the bench line); -1: BoomerAMG's default hybrid "
                         "Gauss-Seidel 13/14 with the automatic block count")
    ap.add_argument("--coarsen", type=int, choices=[8, 10], default=8, help="8: PMIS (the bench line), 10: HMIS")
    ap.add_argument("--cpu-cycles", type=int, default=1, help="run the CPU baseline (0 = skip)")
    ap.add_argument("--parity-iters", type=int, default=8,
                    help="solve iterations from x = 0 that the CPU baseline times and the parity checks compare "
                         "(N = 1: GPU vs the C oracle, bitwise, plus the slab digests; N > 1: the rank slabs' "
                         "sha256 against the N = 1 digests)")
    ap.add_argument("--spmv-reps", type=int, default=50)
    ap.add_argument("--pcg-iters", type=int, default=4,
                    help="one GPU: configs[2]'s BoomerAMG-PCG on the bench hierarchy for this many iterations, "
                         "against the C oracle (parity_pcg; 0 = skip)")
    ap.add_argument("--setup-parity", type=int, default=1,
                    help="one GPU: device setup vs host setup at the secondary size (setup_parity; 0 = skip)")
    ap.add_argument("--calib", action="store_true",
                    help="also run 512 MiB read streams of 2/4/8-B elements (PMC FETCH_SIZE calibration)")
    ap.add_argument("--solver", choices=["amg", "pcg"], default="amg",
                    help="amg: a step is one BoomerAMG solve iteration (the metric); pcg: one PCG iteration "
                         "preconditioned by one V-cycle (configs[2], reported separately)")
    ap.add_argument("--dist", action="store_true",
                    help="take the torch.distributed + RCCL path even with one rank (rehearses the multi-GPU "
                         "launch on a one-GPU box: a 1-rank RCCL communicator, partitioned solve path)")
    ap.add_argument("--loopback", type=int, default=0,
                    help="rehearsal only: N virtual ranks (threads) sharing this process's GPU")
    ap.add_argument("--iters-tol", type=float, default=1e-8,
                    help="one GPU: iterations to this relative residual from x = 0 (V-cycle and PCG), with the C "
                         "oracle's counts at the secondary size (0 = skip)")
    ap.add_argument("--gs-n", type=int, default=256,
                    help="one GPU: also time BoomerAMG's default smoothers (hybrid GS 13 down / 14 up) at this "
                         "size, bitwise against the C oracle (secondary_gs; 0 = skip)")
    ap.add_argument("--emulate", type=int, default=0,
                    help="one GPU: the reference of an N-rank line (the N-rank setup under the rank emulation, "
                         "the iterate checked against the C oracle, its slab digests); no timing")
    args = ap.parse_args()
    if args.emulate > 1:
        rank_threads()
        import hypreve as hv
        sys.exit(emulated_reference(hv, args, args.emulate))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ and args.loopback <= 1:
        # one process per GPU: start the ranks under torch.distributed.run as a
        # child process (nothing here has touched the GPU) and exit with its code
        import subprocess
        ndev = visible_gpus()
        if ndev < args.gpus:
            log(f"[bench] --gpus {args.gpus} needs {args.gpus} GPUs on this node, found {ndev}")
            sys.exit(2)
        import socket
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
        log(f"[bench] launching {args.gpus} ranks: {' '.join(cmd)}")
        sys.exit(subprocess.call(cmd))
    omp = rank_threads()

    import torch  # loads the HIP runtime the library then shares

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.loopback <= 1 and world != args.gpus:
        log(f"[bench] --gpus {args.gpus} but the launcher started {world} rank(s)")
        sys.exit(2)

    import hypreve as hv

    if args.loopback > 1:
        import threading

        torch.cuda.set_device(0)
        hv.init()
        nv = args.loopback
        comms = hv.Comm.loopback(nv)
        bar = threading.Barrier(nv)
        times = [0.0] * nv
        results, errs = [None] * nv, [None] * nv

        slots = [None] * nv

        def worker(r):
            def max_fn(t):
                times[r] = t
                bar.wait()
                return max(times)

            def gather_fn(obj):
                slots[r] = obj
                bar.wait()
                out = list(slots)
                bar.wait()
                return out
            try:
                results[r] = run_rank(hv, args, comms[r], r, nv, bar.wait, max_fn, gather_fn)
            except BaseException as e:
                errs[r] = e
                bar.abort()

        th = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(nv)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        for e in errs:
            if e is not None:
                raise e
        out = results[0]
        out["data"] += f"; LOOPBACK REHEARSAL: {nv} virtual ranks on one GPU (not a multi-GPU measurement)"
        print(json.dumps(out), flush=True)
        return

    dist = None
    comm = None
    if world > 1 or args.dist:
        import torch.distributed as dist

        torch.cuda.set_device(local_rank)
        dist.init_process_group("gloo")
        hv.init()
        uid = hv.Comm.unique_id() if rank == 0 else bytes(128)
        t = torch.tensor(list(uid), dtype=torch.uint8)
        dist.broadcast(t, 0)
        comm = hv.Comm.create(rank, world, bytes(t.tolist()))
    else:
        torch.cuda.set_device(0)
        hv.init()

    def barrier():
        if dist:
            dist.barrier()

    def max_over_ranks(v):
        if not dist:
            return v
        tt = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt.item())

    def gather(obj):
        if not dist:
            return [obj]
        out = [None] * world
        dist.all_gather_object(out, obj)
        return out

    log(f"[bench] rank {rank}/{world}: OpenMP {omp} host threads for the setup")
    out = run_rank(hv, args, comm, rank, world, barrier, max_over_ranks, gather)
    if out is not None and world == 1 and comm is None and args.secondary_n > 0 and args.secondary_n != args.n \
            and not args.grid:
        sec = run_rank(hv, args, None, 0, 1, barrier, max_over_ranks, gather, n=args.secondary_n, light=True)
        out["secondary"] = {k: sec[k] for k in ("value", "unit", "ms_per_step", "steps", tol_key(args.iters_tol))
                            if k in sec}
        out["secondary"]["config"] = sec["config"]
        out["secondary"]["roofline"] = {k: sec["roofline"][k] for k in ("achieved", "frac", "avg_ms", "kernel",
                                                                        "bytes_per_launch", "per_kernel")}
        if args.setup_parity:
            out["setup_parity"] = setup_parity(hv, args, args.secondary_n)
    if out is not None and world == 1 and comm is None and args.gs_n > 0 and not args.grid and args.relax >= 0:
        out["secondary_gs"] = gs_leg(hv, args, args.gs_n)
    if out is not None:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
