"""Partitioned (multi-rank) solve path on one GPU through the loopback hub.

RCCL refuses two ranks on one device, so the N-rank data path -- the
distributed setup (dsetup.cpp) or the rank-0 gathered one, row-block
ownership per level, [local | halo] operators split into interior / boundary
rows, halo exchange on the side stream, redundant coarse solve after a sum
over ranks -- runs here as N virtual ranks, one host thread each, on the box's
single GPU.

One contract for every N-rank run: hypre's own setup on N processes (per-rank
PMIS streams, ParCSR row order, truncation over [P_diag | P_offd], ...), which
hypreve_BoomerAMGSetRankEmulation restates in one process and the
reference's saved np > 1 runs pin (tests/test_reference_pins.py).  So the
N-rank iterates must equal a one-GPU run under the rank emulation with the
same row starts bit for bit (every row sum keeps the stored ParCSR entry
order); only the residual norms may differ in the last bits (the inner
product is summed over ranks in another order), so the iteration counts must
agree.  test_loopback_reference_np_runs takes the reference's own np > 1 runs
through the distributed setup and the partitioned cycle, no emulation, and
prints the saved numbers.  The production transport (RCCL, one process per
GPU) shares all of this code except DevComm::exchange / allreduce_sum.
"""
import threading

import numpy as np
import pytest

import ij_emul
from test_reference_pins import CASES

pytestmark = pytest.mark.gpu


def _slab_starts(nx, ny, nz, nranks):
    """Level-0 row starts of GenerateLaplacian's 1 x 1 x nranks process grid
    (hypre_GeneratePartitioning: the first nz % nranks slabs one plane more)."""
    zp = ij_emul.partition(nz, nranks)
    return [z * nx * ny for z in zp]


def _gen(hv, stencil, nx, ny, nz, **part):
    if stencil == 27:
        return hv.ParCSRMatrix.laplacian27(nx, ny, nz, **part)
    return hv.ParCSRMatrix.laplacian(nx, ny, nz, **part)


def _solve_1rank(hv, nx, ny, nz, kw, stencil=7, nranks=1):
    """One GPU; nranks > 1: the setup of an nranks-process run in z-slabs
    (hypreve_BoomerAMGSetRankEmulation, hybrid-GS blocks included)."""
    A = _gen(hv, stencil, nx, ny, nz)
    amg = hv.BoomerAMG(**kw)
    if nranks > 1:
        amg.set_rank_emulation(_slab_starts(nx, ny, nz, nranks))
    amg.setup(A)
    b = hv.ParVector(A.n, np.ones(A.n))
    x = hv.ParVector(A.n, np.zeros(A.n))
    it, rr = amg.solve(A, b, x)
    return x.get(), it, rr, amg.num_levels()


def _solve_nranks(hv, nx, ny, nz, kw, nranks, timeout=300, stencil=7):
    comms = hv.Comm.loopback(nranks)
    out, errs, paths = [None] * nranks, [None] * nranks, [None] * nranks

    def worker(r):
        try:
            c = comms[r]
            A = _gen(hv, stencil, nx, ny, nz, comm=c, P=1, Q=1, R=nranks, p=0, q=0, r=r)
            amg = hv.BoomerAMG(**kw)
            amg.setup(A)
            b = hv.ParVector(A.n, np.ones(A.n), comm=c, first=A.first, global_n=A.global_n)
            x = hv.ParVector(A.n, np.zeros(A.n), comm=c, first=A.first, global_n=A.global_n)
            it, rr = amg.solve(A, b, x)
            out[r] = (A.first, x.get(), it, rr, amg.num_levels())
            paths[r] = amg.setup_path()
        except Exception as e:  # reported by the main thread
            errs[r] = e

    th = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout)
    assert not any(t.is_alive() for t in th), "a virtual rank did not finish (exchange mismatch?)"
    for e in errs:
        if e is not None:
            raise e
    out.sort(key=lambda o: o[0])
    x = np.concatenate([o[1] for o in out])
    _solve_nranks.starts = [o[0] for o in out] + [x.size]  # level-0 row starts of the run
    _solve_nranks.paths = paths
    return x, [o[2] for o in out], [o[3] for o in out], out[0][4]


@pytest.mark.parametrize("nranks,nx,nz", [(2, 16, 16), (3, 14, 20), (4, 12, 13)])
@pytest.mark.parametrize("agglo", [0, 2000])
@pytest.mark.parametrize("relax", [18, 0, 17])
def test_loopback_partitioned_solve_bitwise(hv, nranks, nx, nz, relax, agglo):
    """agglo 0: every level distributed; 2000: the coarse levels from the first
    one under 2000 rows are replicated on every rank (one all-gather down).
    The distributed setup takes these options; its hierarchy is the rank
    emulation's, and the one-process hierarchy is not."""
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=relax, tol=1e-8, max_iter=60, agglo_rows=agglo)
    if relax == 0:
        kw.update(relax_wt=0.6)
    x1, it1, rr1, nl1 = _solve_1rank(hv, nx, nx, nz, kw, nranks=nranks)
    xN, itN, rrN, nlN = _solve_nranks(hv, nx, nx, nz, kw, nranks)
    assert _solve_nranks.paths == ["distributed"] * nranks
    assert _solve_nranks.starts == _slab_starts(nx, nx, nz, nranks)
    assert nlN == nl1
    assert all(i == it1 for i in itN), (it1, itN)
    assert all(abs(r - rr1) <= 1e-10 * rr1 for r in rrN), (rr1, rrN)
    assert x1.shape == xN.shape
    assert np.array_equal(x1, xN), f"max |diff| {np.max(np.abs(x1 - xN))}"
    if relax == 18 and agglo == 0:
        # the contract has teeth: the one-process setup (one PMIS stream, global
        # entry order) is another hierarchy, hence another iterate
        xp, _, _, _ = _solve_1rank(hv, nx, nx, nz, kw)
        assert not np.array_equal(xp, xN)


@pytest.mark.parametrize("nranks,nx,nz", [(2, 14, 16), (3, 12, 17)])
@pytest.mark.parametrize("relax,order", [(3, 0), (6, 0), (13, 0), (8, 1)])
@pytest.mark.parametrize("nb", [1, 3])
@pytest.mark.parametrize("agglo", [0, 2000])
def test_loopback_hybrid_gs_bitwise(hv, nranks, nx, nz, relax, order, nb, agglo):
    """Hybrid Gauss-Seidel across ranks (par_relax.c with num_procs > 1): each
    rank sweeps its rows in num_blocks blocks, off-rank columns read the halo
    exchanged before the sweep, off-block columns the pre-sweep copy, and the
    l1 norms (relax 8/13) follow those blocks, on the agglomerated levels too.
    One GPU under the rank emulation (its GS blocks are the ranks' blocks) must
    reproduce the N-rank iterates bit for bit; relax 8 with C/F ordering
    exchanges once per point class, as hypre's two relax calls do."""
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=relax, relax_order=order, num_blocks=nb,
              tol=1e-8, max_iter=40, agglo_rows=agglo)
    xN, itN, rrN, nlN = _solve_nranks(hv, nx, nx, nz, kw, nranks)
    x1, it1, rr1, nl1 = _solve_1rank(hv, nx, nx, nz, kw, nranks=nranks)
    assert nlN == nl1
    assert all(i == it1 for i in itN), (it1, itN)
    assert np.array_equal(x1, xN), f"max |diff| {np.max(np.abs(x1 - xN))}"
    if nb == 1 and agglo == 0 and relax == 3:
        # control: the same rank setup with one GPU's own blocks is another smoother
        A = _gen(hv, 7, nx, nx, nz)
        amg = hv.BoomerAMG(**kw)
        amg.set_rank_emulation(_solve_nranks.starts)
        amg.set_gs_rank_starts(None)
        amg.setup(A)
        b = hv.ParVector(A.n, np.ones(A.n))
        x = hv.ParVector(A.n, np.zeros(A.n))
        amg.solve(A, b, x)
        assert not np.array_equal(x.get(), xN)


@pytest.mark.parametrize("nranks", [2, 3])
def test_loopback_partitioned_27pt(hv, nranks):
    """27-point operator (configs[3]'s stencil), z-slab row blocks."""
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=18, tol=1e-8, max_iter=60)
    x1, it1, rr1, nl1 = _solve_1rank(hv, 13, 12, 15, kw, stencil=27, nranks=nranks)
    xN, itN, rrN, nlN = _solve_nranks(hv, 13, 12, 15, kw, nranks, stencil=27)
    assert nlN == nl1 and all(i == it1 for i in itN)
    assert np.array_equal(x1, xN)


@pytest.mark.parametrize("nranks", [2, 3])
def test_loopback_comm_selftest(hv, nranks):
    """Every transport operation the solve uses, checked value by value."""
    hv.init()
    comms = hv.Comm.loopback(nranks)
    errs = [None] * nranks

    def worker(r):
        try:
            comms[r].self_test()
        except Exception as e:
            errs[r] = e

    th = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not any(t.is_alive() for t in th)
    assert errs == [None] * nranks, errs


def test_rccl_single_rank(hv):
    """The production transport on a one-GPU box: a 1-rank RCCL communicator
    (RCCL refuses two ranks on one device).  The self-test sends to its own
    rank through ncclGroupStart/Send/Recv/GroupEnd and runs ncclAllReduce;
    then a BoomerAMG solve over that communicator takes the partitioned path
    (rank-0 setup shipped over RCCL, dots summed by ncclAllReduce) and must
    reproduce the communicator-free solve bit for bit."""
    hv.init()
    c = hv.Comm.create(0, 1, hv.Comm.unique_id())
    c.self_test()
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=8, relax_type=18, tol=1e-8, max_iter=60)
    x1, it1, rr1, nl1 = _solve_1rank(hv, 20, 18, 16, kw)
    A = hv.ParCSRMatrix.laplacian(20, 18, 16, comm=c, P=1, Q=1, R=1, p=0, q=0, r=0)
    amg = hv.BoomerAMG(**kw)
    amg.setup(A)
    b = hv.ParVector(A.n, np.ones(A.n), comm=c, first=A.first, global_n=A.global_n)
    x = hv.ParVector(A.n, np.zeros(A.n), comm=c, first=A.first, global_n=A.global_n)
    it, rr = amg.solve(A, b, x)
    assert it == it1
    assert np.array_equal(x.get(), x1)
    assert abs(rr - rr1) <= 1e-10 * rr1


@pytest.mark.parametrize("nranks", [2, 3])
def test_loopback_aggressive_bitwise(hv, nranks):
    """Aggressive levels on the multi-rank path (the distributed setup: second
    PMIS pass and multipass interpolation across ranks): the N-rank iterates
    equal the one-rank ones."""
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=18, tol=1e-8, max_iter=80,
              agg_num_levels=1)
    x1, it1, rr1, nl1 = _solve_1rank(hv, 16, 16, 18, kw, nranks=nranks)
    xN, itN, rrN, nlN = _solve_nranks(hv, 16, 16, 18, kw, nranks)
    assert nlN == nl1 and all(i == it1 for i in itN)
    assert np.array_equal(x1, xN)


@pytest.mark.parametrize("nranks", [2, 3])
@pytest.mark.parametrize("stencil,relax", [(7, 18), (7, 0), (27, 18)])
def test_loopback_stencil_layout_bitwise(hv, nranks, stencil, relax):
    """The slot-uniform stencil layout (policy 11) on the interior and boundary
    rows of every rank's finest operator: offsets are taken from the stored
    row, so a rank's interior rows (one plane in) keep one offset per slot.
    The N-rank iterates equal the one-rank ones, and both use the layout."""
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=relax, tol=1e-8, max_iter=60,
              sell_policy=11)
    if relax == 0:
        kw.update(relax_wt=0.6)
    x1, it1, rr1, nl1 = _solve_1rank(hv, 14, 13, 16, kw, stencil=stencil, nranks=nranks)
    xN, itN, rrN, nlN = _solve_nranks(hv, 14, 13, 16, kw, nranks, stencil=stencil)
    assert nlN == nl1 and all(i == it1 for i in itN)
    assert np.array_equal(x1, xN)


@pytest.mark.parametrize("nranks", [2, 3])
@pytest.mark.parametrize("agglo", [0, 20000])
def test_loopback_coded_layout_bitwise(hv, nranks, agglo):
    """Offset-coded P and R (policy 12) on every rank's interior rows: anchors
    and the fine -> coarse map are rank-local, boundary rows and the
    agglomerated levels keep the other layouts.  The N-rank iterates equal the
    one-rank ones bit for bit."""
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=18, tol=1e-8, max_iter=60,
              sell_policy=12, agglo_rows=agglo)
    x1, it1, rr1, nl1 = _solve_1rank(hv, 14, 13, 16, kw, nranks=nranks)
    xN, itN, rrN, nlN = _solve_nranks(hv, 14, 13, 16, kw, nranks)
    assert nlN == nl1 and all(i == it1 for i in itN)
    assert np.array_equal(x1, xN)


@pytest.mark.parametrize("nranks", [2, 3])
@pytest.mark.parametrize("stencil,relax", [(7, 18), (27, 18), (7, 0)])
def test_loopback_grid_stencil_bitwise(hv, nranks, stencil, relax):
    """The grid-stencil loop (k_grid_stencil) on every rank's interior rows:
    a run of whole planes one plane in from the slab's faces, read as grid
    points shifted by that plane.  The N-rank iterates equal the one-rank ones
    bit for bit, and every rank's interior operator takes the grid form."""
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=relax, tol=1e-8, max_iter=60,
              sell_policy=11)
    if relax == 0:
        kw.update(relax_wt=0.6)
    x1, it1, rr1, nl1 = _solve_1rank(hv, 64, 20, 24, kw, stencil=stencil, nranks=nranks)
    comms = hv.Comm.loopback(nranks)
    layouts, out, errs = [None] * nranks, [None] * nranks, [None] * nranks

    def worker(r):
        try:
            c = comms[r]
            A = _gen(hv, stencil, 64, 20, 24, comm=c, P=1, Q=1, R=nranks, p=0, q=0, r=r)
            amg = hv.BoomerAMG(**kw)
            amg.setup(A)
            layouts[r] = amg.level_layout(0, 0)
            b = hv.ParVector(A.n, np.ones(A.n), comm=c, first=A.first, global_n=A.global_n)
            x = hv.ParVector(A.n, np.zeros(A.n), comm=c, first=A.first, global_n=A.global_n)
            it, rr = amg.solve(A, b, x)
            out[r] = (A.first, x.get(), it)
        except Exception as e:  # reported by the main thread
            errs[r] = e

    th = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join(300)
    assert not any(t.is_alive() for t in th), "a virtual rank did not finish"
    for e in errs:
        if e is not None:
            raise e
    assert all(lay == "grid-stencil" for lay in layouts), layouts
    out.sort(key=lambda o: o[0])
    xN = np.concatenate([o[1] for o in out])
    assert all(o[2] == it1 for o in out)
    assert np.array_equal(x1, xN)


@pytest.mark.parametrize("nranks,nx,nz", [(2, 16, 16), (3, 14, 20)])
@pytest.mark.parametrize("relax,interp,agg", [(18, 6, 0), (13, 6, 0), (18, 14, 0), (18, 6, 1)])
def test_loopback_hmis_bitwise(hv, nranks, nx, nz, relax, interp, agg):
    """HMIS (hypre's default coarsening) set up distributed across the ranks
    (each rank's Ruge first pass, PMIS with per-rank streams; dsetup.cpp
    hmis_dist) and solved: one GPU under the rank emulation with the same
    starts reproduces the N-rank iterates bit for bit."""
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=10, interp_type=interp, P_max_elmts=4, relax_type=relax, tol=1e-8, max_iter=40,
              agg_num_levels=agg)
    xN, itN, rrN, nlN = _solve_nranks(hv, nx, nx, nz, kw, nranks)
    assert _solve_nranks.paths == ["distributed"] * nranks
    x1, it1, rr1, nl1 = _solve_1rank(hv, nx, nx, nz, kw, nranks=nranks)
    assert nlN == nl1
    assert all(i == it1 for i in itN), (it1, itN)
    assert np.array_equal(x1, xN), f"max |diff| {np.max(np.abs(x1 - xN))}"


# The reference's own np > 1 runs (TEST_ij/*.saved, tests/golden/ij_rank_fixtures.json)
# whose options the distributed setup takes: PMIS (8), PMIS1 (9) and HMIS (10),
# ext+i with Pmx 0 / 4, the 7- and 27-point operators, relax 0 / 18 (C/F-ordered
# too), hybrid GS 6 / 8 under PCG, an aggressive level with multipass
# interpolation.  -P process grids in x and y as well as z.
LOOPBACK_PINS = ["coarsening.out.4", "coarsening.out.13", "default.out.1", "interp.out.3", "matrix.out.0",
                 "smoother.out.9", "smoother.out.10", "solvers.out.0", "smoother.out.11", "agg_interp.out.4"]


# seq_threshold (the redundant coarse-grid AMG, gen_redcs_mat.c) takes the
# gathered setup, which runs the rank emulation on rank 0
GATHERED_PINS = ["solvers.out.105", "solvers.out.106"]


@pytest.mark.parametrize("name", LOOPBACK_PINS)
def test_loopback_reference_np_runs(hv, name):
    """A reference `mpirun -np N ./ij ...` run, N loopback ranks, no emulation:
    every rank generates its block of the -P process grid
    (GenerateLaplacian[27pt], rank = p + P q + P Q r), sets up its own rows
    through the distributed setup (dsetup.cpp: per-rank PMIS streams, ParCSR
    row order, truncation over [P_diag | P_offd], ...), and solves through the
    partitioned cycle (halo exchange, agglomerated coarse levels).  The saved
    iteration count and final relative residual, or convergence factor and
    complexities, come out to every printed digit."""
    _loopback_pin(hv, name, "distributed")


@pytest.mark.parametrize("name", GATHERED_PINS)
def test_loopback_reference_gathered_runs(hv, name):
    """The same for 8-rank runs with seq_threshold 100 (solvers.out.105 / 106,
    80^3, aggressive level, hybrid GS 6 under PCG): the ranks gather to rank 0,
    whose setup is hypre's 8-process one (the rank emulation) with the
    one-process BoomerAMG below 100 rows appended, and the partitioned cycle
    reproduces the saved iterations and residual on every rank."""
    _loopback_pin(hv, name, "gathered, rank emulation")


def _loopback_pin(hv, name, path):
    case = next(c for c in CASES if c["name"] == name)
    prob = case["problem"]
    P, Q, R = prob["P"]
    nx, ny, nz = prob["n"]
    nranks = P * Q * R
    pt27 = prob["stencil"] == 27
    A_s, starts = ij_emul.laplacian_ranks(nx, ny, nz, P, Q, R, pt27=pt27)
    if case["rhs"] == "rhsrand":
        b_glob = ij_emul.rhsrand(starts)
    elif case["rhs"] == "xisone":
        b_glob = A_s @ np.ones(A_s.shape[0])
    else:
        b_glob = np.ones(A_s.shape[0])
    pcg_run = case["solver"] == "pcg"
    kw = hv.ij_amg_defaults(1 if pcg_run else 0)
    kw.update(num_blocks=1)
    kw.update(case["settings"])
    comms = hv.Comm.loopback(nranks)
    out, errs = [None] * nranks, [None] * nranks

    def worker(rk):
        try:
            c = comms[rk]
            p, q, r = rk % P, (rk // P) % Q, rk // (P * Q)
            part = dict(comm=c, P=P, Q=Q, R=R, p=p, q=q, r=r)
            A = hv.ParCSRMatrix.laplacian27(nx, ny, nz, **part) if pt27 else hv.ParCSRMatrix.laplacian(nx, ny, nz, **part)
            assert A.first == starts[rk] and A.n == starts[rk + 1] - starts[rk], (rk, A.first, A.n)
            gn = A_s.shape[0]
            b = hv.ParVector(A.n, b_glob[A.first:A.first + A.n], comm=c, first=A.first, global_n=gn)
            x = hv.ParVector(A.n, np.zeros(A.n), comm=c, first=A.first, global_n=gn)
            amg = hv.BoomerAMG(**kw)
            if pcg_run:
                pcg = hv.PCG(tol=1e-8, max_iter=1000, two_norm=1)
                pcg.set_precond_amg(amg)
                pcg.setup(A, b, x)
                it, rr = pcg.solve(A, b, x)
                pcg.destroy()
            else:
                amg.setup(A)
                it, rr = amg.solve(A, b, x)
            out[rk] = (it, rr, amg.complexities(), amg.setup_path())
        except Exception as e:  # reported by the main thread
            errs[rk] = e

    th = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join(300)
    assert not any(t.is_alive() for t in th), "a virtual rank did not finish"
    for e in errs:
        if e is not None:
            raise e
    # the gathered setup records its path on rank 0 (the others receive levels)
    assert out[0][3] == path and all(o[3] in (path, None) for o in out), [o[3] for o in out]
    it, rr, (g, o, cyc), _ = out[0]
    assert all(ob[0] == it for ob in out)
    exp = case["expect"]
    print(name, case["cmd"], "->", it, f"{rr:e}", f"conv {rr ** (1.0 / it):f}", f"grid {g:f} op {o:f} cycle {cyc:f}")
    if "iterations" in exp:
        assert it == exp["iterations"]
        assert f"{rr:e}" == f"{exp['rel_res']:e}"
    if "conv_factor" in exp:  # ij's "Average Convergence Factor": (|r_k| / |r_0|)^(1/k), x0 = 0
        assert f"{rr ** (1.0 / it):f}" == f"{exp['conv_factor']:f}"
    if "grid" in exp:
        assert f"{g:f}" == f"{exp['grid']:f}"
        assert f"{o:f}" == f"{exp['operator']:f}"
        assert abs(cyc - exp["cycle"]) < 1.5e-6
