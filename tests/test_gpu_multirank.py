"""Partitioned (multi-rank) solve path on one GPU through the loopback hub.

RCCL refuses two ranks on one device, so the N-rank data path -- row-block
ownership per level, [local | halo] operators split into interior / boundary
rows, halo exchange on the side stream, rank-0 setup shipped to every rank,
redundant coarse solve after a sum over ranks -- runs here as N virtual ranks,
one host thread each, on the box's single GPU.  The iterates must equal the
1-rank iterates bit for bit (every row sum keeps the global entry order);
only the residual norms may differ in the last bits (the inner product is
summed over ranks in another order), so the iteration counts must agree.
The production transport (RCCL, one process per GPU) shares all of this code
except DevComm::exchange / allreduce_sum.
"""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _gen(hv, stencil, nx, ny, nz, **part):
    if stencil == 27:
        return hv.ParCSRMatrix.laplacian27(nx, ny, nz, **part)
    return hv.ParCSRMatrix.laplacian(nx, ny, nz, **part)


def _solve_1rank(hv, nx, ny, nz, kw, stencil=7):
    A = _gen(hv, stencil, nx, ny, nz)
    amg = hv.BoomerAMG(**kw)
    amg.setup(A)
    b = hv.ParVector(A.n, np.ones(A.n))
    x = hv.ParVector(A.n, np.zeros(A.n))
    it, rr = amg.solve(A, b, x)
    return x.get(), it, rr, amg.num_levels()


def _solve_nranks(hv, nx, ny, nz, kw, nranks, timeout=300, stencil=7):
    comms = hv.Comm.loopback(nranks)
    out, errs = [None] * nranks, [None] * nranks

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
    return x, [o[2] for o in out], [o[3] for o in out], out[0][4]


@pytest.mark.parametrize("nranks,nx,nz", [(2, 16, 16), (3, 14, 20), (4, 12, 13)])
@pytest.mark.parametrize("agglo", [0, 2000])
@pytest.mark.parametrize("relax", [18, 0, 17])
def test_loopback_partitioned_solve_bitwise(hv, nranks, nx, nz, relax, agglo):
    """agglo 0: every level distributed; 2000: the coarse levels from the first
    one under 2000 rows are replicated on every rank (one all-gather down)."""
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=relax, tol=1e-8, max_iter=60, agglo_rows=agglo)
    if relax == 0:
        kw.update(relax_wt=0.6)
    x1, it1, rr1, nl1 = _solve_1rank(hv, nx, nx, nz, kw)
    xN, itN, rrN, nlN = _solve_nranks(hv, nx, nx, nz, kw, nranks)
    assert nlN == nl1
    assert all(i == it1 for i in itN), (it1, itN)
    assert all(abs(r - rr1) <= 1e-10 * rr1 for r in rrN), (rr1, rrN)
    assert x1.shape == xN.shape
    assert np.array_equal(x1, xN), f"max |diff| {np.max(np.abs(x1 - xN))}"


@pytest.mark.parametrize("nranks,nx,nz", [(2, 14, 16), (3, 12, 17)])
@pytest.mark.parametrize("relax,order", [(3, 0), (6, 0), (13, 0), (8, 1)])
@pytest.mark.parametrize("nb", [1, 3])
@pytest.mark.parametrize("agglo", [0, 2000])
def test_loopback_hybrid_gs_bitwise(hv, nranks, nx, nz, relax, order, nb, agglo):
    """Hybrid Gauss-Seidel across ranks (par_relax.c with num_procs > 1): each
    rank sweeps its rows in num_blocks blocks, off-rank columns read the halo
    exchanged before the sweep, off-block columns the pre-sweep copy, and the
    l1 norms (relax 8/13) follow those blocks.  One GPU given the same row
    blocks (hypreve_BoomerAMGSetGsRankStarts) must reproduce the N-rank
    iterates bit for bit; relax 8 with C/F ordering exchanges once per
    point class, as hypre's two relax calls do."""
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=relax, relax_order=order, num_blocks=nb,
              tol=1e-8, max_iter=40, agglo_rows=agglo)
    xN, itN, rrN, nlN = _solve_nranks(hv, nx, nx, nz, kw, nranks)
    starts = _solve_nranks.starts
    A = _gen(hv, 7, nx, nx, nz)
    amg = hv.BoomerAMG(**kw)
    amg.set_gs_rank_starts(starts)
    amg.setup(A)
    b = hv.ParVector(A.n, np.ones(A.n))
    x = hv.ParVector(A.n, np.zeros(A.n))
    it1, rr1 = amg.solve(A, b, x)
    x1 = x.get()
    assert nlN == amg.num_levels()
    assert all(i == it1 for i in itN), (it1, itN)
    assert np.array_equal(x1, xN), f"max |diff| {np.max(np.abs(x1 - xN))}"
    if nb == 1 and agglo == 0 and relax == 3:
        # control: without the rank blocks one GPU runs a different smoother
        xp, _, _, _ = _solve_1rank(hv, nx, nx, nz, kw)
        assert not np.array_equal(xp, xN)


@pytest.mark.parametrize("nranks", [2, 3])
def test_loopback_partitioned_27pt(hv, nranks):
    """27-point operator (configs[3]'s stencil), z-slab row blocks."""
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=18, tol=1e-8, max_iter=60)
    x1, it1, rr1, nl1 = _solve_1rank(hv, 13, 12, 15, kw, stencil=27)
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
    x1, it1, rr1, nl1 = _solve_1rank(hv, 16, 16, 18, kw)
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
    x1, it1, rr1, nl1 = _solve_1rank(hv, 14, 13, 16, kw, stencil=stencil)
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
    x1, it1, rr1, nl1 = _solve_1rank(hv, 14, 13, 16, kw)
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
    x1, it1, rr1, nl1 = _solve_1rank(hv, 64, 20, 24, kw, stencil=stencil)
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
    hmis_dist) and solved: one GPU given the same rank starts for the
    coarsening (hypreve_BoomerAMGSetCoarsenRankStarts; hybrid GS: the rank
    blocks too) reproduces the N-rank iterates bit for bit."""
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=10, interp_type=interp, P_max_elmts=4, relax_type=relax, tol=1e-8, max_iter=40,
              agg_num_levels=agg)
    xN, itN, rrN, nlN = _solve_nranks(hv, nx, nx, nz, kw, nranks)
    starts = _solve_nranks.starts
    A = _gen(hv, 7, nx, nx, nz)
    amg = hv.BoomerAMG(**kw)
    amg.set_coarsen_rank_starts(starts)
    if relax == 13:
        amg.set_gs_rank_starts(starts)
    amg.setup(A)
    b = hv.ParVector(A.n, np.ones(A.n))
    x = hv.ParVector(A.n, np.zeros(A.n))
    it1, rr1 = amg.solve(A, b, x)
    x1 = x.get()
    assert nlN == amg.num_levels()
    assert all(i == it1 for i in itN), (it1, itN)
    assert np.array_equal(x1, xN), f"max |diff| {np.max(np.abs(x1 - xN))}"
