"""Host setup logic: determinism across thread counts, structural invariants."""
import hashlib
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_SCRIPT = r"""
import sys, hashlib, numpy as np
sys.path.insert(0, %r)
import hypreve as hv
A = hv.ParCSRMatrix.laplacian(24, 22, 20)
amg = hv.BoomerAMG(**hv.ij_amg_defaults(0)); amg.set(coarsen_type=int(sys.argv[1]), relax_type=18, P_max_elmts=4)
amg.setup_host(A)
h = hashlib.sha256()
for l in range(amg.num_levels()):
    for w in (0, 1):
        ip, jj, vv, shp = amg.level_matrix(l, w)
        for a in (ip, jj, vv): h.update(np.ascontiguousarray(a).tobytes())
    h.update(amg.level_vector(l, 0).tobytes()); h.update(amg.level_vector(l, 1).tobytes())
print(h.hexdigest())
""" % os.path.join(ROOT, "hypre-ve_amd")


def _digest(threads, coarsen_type):
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    out = subprocess.run([sys.executable, "-c", _SCRIPT, str(coarsen_type)], env=env, capture_output=True,
                         text=True, check=True)
    return out.stdout.strip()


@pytest.mark.parametrize("coarsen_type", [8, 10, 11])
def test_setup_bitwise_independent_of_threads(coarsen_type):
    d1 = _digest(1, coarsen_type)
    assert d1 == _digest(3, coarsen_type) == _digest(8, coarsen_type)


@pytest.mark.parametrize("coarsen_type", [8, 10, 11])
def test_hierarchy_invariants(hv, coarsen_type):
    A = hv.ParCSRMatrix.laplacian(16, 16, 16)
    amg = hv.BoomerAMG(**hv.ij_amg_defaults(0))
    amg.set(coarsen_type=coarsen_type, relax_type=18, P_max_elmts=4)
    amg.setup_host(A)
    nl = amg.num_levels()
    assert nl >= 3
    import scipy.sparse as sp
    for l in range(nl - 1):
        ip, jj, vv, shp = amg.level_matrix(l, 0)
        Al = sp.csr_matrix((vv, jj, ip), shape=shp)
        # diagonal stored first in every row (hypre ParCSR convention)
        assert np.all(jj[ip[:-1]] == np.arange(shp[0]))
        ip, jj, vv, pshp = amg.level_matrix(l, 1)
        P = sp.csr_matrix((vv, jj, ip), shape=pshp)
        assert np.all(np.diff(ip) <= 4)  # P_max_elmts
        cf = amg.level_vector(l, 0)
        # C points interpolate by injection
        c = np.where(cf == 1)[0]
        assert np.allclose(P[c].toarray().max(axis=1), 1.0)
        assert set(np.unique(cf)) <= {1, -1, -3}
        # every F point with strong connections has a strong C neighbour
        # (PMIS / HMIS second phase; the Ruge first pass on a symmetric S); on
        # these M-matrices every off-diagonal entry is strong at threshold 0.25
        # unless the row sum test drops it
        Aoff = Al.copy(); Aoff.setdiag(0); Aoff.eliminate_zeros()
        fpts = np.where(cf == -1)[0]
        hasC = (abs(Aoff[fpts]) @ (cf == 1).astype(float)) > 0
        assert hasC.all()
        ip, jj, vv, cshp = amg.level_matrix(l + 1, 0)
        Ac = sp.csr_matrix((vv, jj, ip), shape=cshp)
        # Galerkin: A_c == P^T A P (values; order of summation may differ slightly)
        G = (P.T @ Al @ P).tocsr()
        assert abs(G - Ac).max() < 1e-12 * abs(Ac).max()
        # symmetric
        assert abs(Ac - Ac.T).max() < 1e-12 * abs(Ac).max()
        # l1 norms (relax 18): row sums of |a|
        l1 = amg.level_vector(l, 1)
        assert np.allclose(l1, abs(Al).sum(axis=1).A1, rtol=1e-14)


def test_partition_self_check(hv):
    """Row partition over N ranks: every rank's interior+boundary operators on
    [local | halo] vectors reproduce the global operators row for row (bitwise),
    and the pairwise halo send/recv plans agree."""
    A = hv.ParCSRMatrix.laplacian(20, 18, 24)
    for agglo in (0, 2000, 20000):
        amg = hv.BoomerAMG(**hv.ij_amg_defaults(0))
        amg.set(coarsen_type=8, relax_type=18, P_max_elmts=4, agglo_rows=agglo)
        amg.setup_host(A)
        for size in (1, 2, 3, 4, 7, 8):
            amg.partition_check(size)


@pytest.mark.parametrize("agglo", [0, 20000])
@pytest.mark.parametrize("size", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("stencil,relax,order", [(7, 18, 0), (7, 0, 1), (27, 18, 0), (7, 13, 0)])
def test_distributed_setup_matches_one_process(hv, size, stencil, relax, order, agglo):
    """Distributed setup (each rank builds its rows' levels from a ghost
    layer: PMIS passes exchanging measures / demotions / C-F state, ext+i over
    fetched neighbour rows, R from P entries sent to their coarse owner, RAP
    over fetched A and P rows) on `size` host threads, under hypre's N-process
    rules (per-rank PMIS streams, rows in ParCSR order, truncation over
    [P_diag | P_offd]): every rank's part of every level equals the rank
    emulation's one-process hierarchy (SetRankEmulation, pinned to the
    reference's np > 1 runs) partitioned the same way, byte for byte
    (operators, C/F, l1 norms, hybrid-GS blocks, halo plans, coarsest operator)."""
    if stencil == 27:
        A = hv.ParCSRMatrix.laplacian27(17, 15, 19)
    else:
        A = hv.ParCSRMatrix.laplacian(19, 17, 23, cx=1.0, cy=0.7 if relax == 0 else 1.0, cz=1.0)
    amg = hv.BoomerAMG(**hv.ij_amg_defaults(0))
    amg.set(coarsen_type=8, interp_type=6, relax_type=relax, relax_order=order, P_max_elmts=4, agglo_rows=agglo)
    amg.dist_setup_check(A, size)


@pytest.mark.parametrize("size", [2, 3, 5])
@pytest.mark.parametrize("agg,cx", [(1, 1.0), (2, 1.0), (1, 0.001), (10, 0.001)])
def test_distributed_setup_aggressive(hv, size, agg, cx):
    """configs[4]: aggressive levels in the distributed setup (second strength
    over the C points from fetched neighbour S rows, PMIS with CF_init 3 and
    per-rank streams, CorrectCFMarker, multipass interpolation pass by pass
    with the previous pass's ghost P rows fetched, rows as P_diag | P_offd)
    equal the rank emulation's hierarchy byte for byte."""
    A = hv.ParCSRMatrix.laplacian(19, 17, 23, cx=cx)
    amg = hv.BoomerAMG(**hv.ij_amg_defaults(0))
    amg.set(coarsen_type=8, interp_type=6, relax_type=18, P_max_elmts=4, agg_num_levels=agg)
    amg.dist_setup_check(A, size)


@pytest.mark.parametrize("size", [2, 4, 7])
def test_distributed_setup_anisotropic(hv, size):
    """configs[4]'s operator family (anisotropic diffusion, strong couplings in
    one direction only): the distributed setup still equals the rank emulation."""
    A = hv.ParCSRMatrix.laplacian(21, 19, 25, cx=0.001, cy=1.0, cz=1.0)
    amg = hv.BoomerAMG(**hv.ij_amg_defaults(0))
    amg.set(coarsen_type=8, interp_type=6, relax_type=18, P_max_elmts=4)
    amg.dist_setup_check(A, size)


@pytest.mark.parametrize("coarsen_type", [8, 10])
def test_gs_level_schedule_matches_sequential_sweep(hv, coarsen_type):
    """Hybrid Gauss-Seidel on the GPU runs each hypre thread block as a level
    schedule (the reference's relax-6 multi-level scheduling, par_relax.c:2340).
    On every level operator, both sweep directions, diagonal (3/4/6) and l1
    (8/13/14) scaling, and several block counts, the level-parallel sweep must
    equal the sequential per-block sweep bit for bit."""
    A = hv.ParCSRMatrix.laplacian(14, 12, 11)
    amg = hv.BoomerAMG(**hv.ij_amg_defaults(0))
    amg.set(coarsen_type=coarsen_type, relax_type=13, P_max_elmts=4)
    amg.setup_host(A)
    for nb in (1, 2, 7, 64, 100000):
        amg.gs_schedule_check(nb)


def test_gs_level_schedule_nonsymmetric(hv):
    """Nonsymmetric pattern: a row may need an un-updated upper neighbour that
    does not depend on it; the schedule must keep that neighbour above it."""
    import scipy.sparse as sp
    rng = np.random.default_rng(11)
    n = 400
    M = sp.random(n, n, density=0.02, random_state=12, format="csr")
    M.data = -np.abs(M.data)
    M = M + sp.diags(np.asarray(abs(M).sum(axis=1)).ravel() + 1.0 + rng.random(n))
    M = M.tocsr()
    M.sort_indices()
    # diagonal first in every row (ParCSR convention)
    rows = []
    for i in range(n):
        cols = list(M.indices[M.indptr[i]:M.indptr[i + 1]])
        vals = list(M.data[M.indptr[i]:M.indptr[i + 1]])
        k = cols.index(i)
        rows.append(([cols[k]] + cols[:k] + cols[k + 1:], [vals[k]] + vals[:k] + vals[k + 1:]))
    ip = np.cumsum([0] + [len(r[0]) for r in rows])
    A = sp.csr_matrix((np.concatenate([r[1] for r in rows]), np.concatenate([r[0] for r in rows]), ip), shape=(n, n))
    A.has_sorted_indices = False
    P = hv.ParCSRMatrix.from_scipy(A)
    amg = hv.BoomerAMG(**hv.ij_amg_defaults(0))
    amg.set(max_levels=1, relax_type=13)
    amg.setup_host(P)
    for nb in (1, 3, 17):
        amg.gs_schedule_check(nb)


@pytest.mark.parametrize("scale", [0, 1])
def test_chebyshev_setup(hv, scale):
    """Relax type 16 setup (par_amg_setup.c:3139): the CG / Lanczos estimate of
    the largest eigenvalue of D^-1/2 A D^-1/2 (or A) from 10 steps lies just
    below the true one (numpy), the smallest above the true smallest, and the
    order-2 coefficients are par_cheby.c's closed form for that interval.
    Parity unpinned: no reference output covers relax 16 at np=1; the
    estimate and the coefficients are restated from par_relax_more.c:115 and
    par_cheby.c:36."""
    import scipy.sparse as sp
    import scipy.sparse.linalg as sla
    A = hv.ParCSRMatrix.laplacian(12, 11, 10)
    amg = hv.BoomerAMG(**hv.ij_amg_defaults(0))
    amg.set(coarsen_type=8, relax_type=16, cheby_scale=scale, cheby_order=2, cheby_fraction=0.3)
    amg.setup_host(A)
    for l in range(amg.num_levels() - 1):
        ip, jj, vv, shp = amg.level_matrix(l, 0)
        M = sp.csr_matrix((vv, jj, ip), shape=shp)
        if scale:
            d = 1.0 / np.sqrt(M.diagonal())
            M = sp.diags(d) @ M @ sp.diags(d)
            assert np.array_equal(amg.level_vector(l, 2), 1 / np.sqrt(sp.csr_matrix((vv, jj, ip), shape=shp).diagonal()))
        lam = np.linalg.eigvalsh(M.toarray()) if shp[0] <= 2000 else sla.eigsh(M, 1, which="LA")[0]
        co, (emax, emin), prm = amg.cheby_info(l)
        assert prm == (2, scale, 0)
        assert emax <= lam.max() * (1 + 1e-10) and emax >= 0.8 * lam.max()
        assert emin >= lam.min() * (1 - 1e-10)
        ub = emax * 1.1
        lb = (ub - emin) * 0.3 + emin
        th, de = (ub + lb) / 2, (ub - lb) / 2
        # order 2 = residual polynomial of degree 2: s(A) of degree 1 (case 1)
        den = de * de - 2 * th * th
        ref = [-4 * th / den, 2 / den, 0.0]
        assert np.allclose(co, ref, rtol=1e-13, atol=0)


@pytest.mark.parametrize("gen,dims,width", [("7", (200, 180, 3), 7), ("7", (10, 10, 10), 7), ("27", (13, 12, 15), 27),
                                             ("aniso", (28, 26, 24), 7), ("7", (1, 1, 70), 3)])
def test_stencil_layout_rebuilds_rows(hv, gen, dims, width):
    """The slot-uniform stencil layout (A0 of constant-coefficient operators):
    every row rebuilt from its slice's slot pattern equals the CSR row entry
    for entry, values bit for bit, the diagonal in slot 0.  (200, 180, 3)
    has slices with no full row (y = 0 and y = 179 lines in one slice: the
    slots are a common supersequence of all its rows); (1, 1, 70) is a 1-D
    chain.  The
    Galerkin level 1 is no stencil: the layout does not build there."""
    if gen == "27":
        A = hv.ParCSRMatrix.laplacian27(*dims)
    elif gen == "aniso":
        A = hv.ParCSRMatrix.laplacian(*dims, cx=0.001, cy=1.0, cz=1.0)
    else:
        A = hv.ParCSRMatrix.laplacian(*dims)
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=18)
    amg = hv.BoomerAMG(**kw)
    amg.setup_host(A)
    w, npat = amg.stencil_layout_check(0)
    assert w == width  # rows in ascending column order merge into the stencil's own slots
    assert 1 <= npat <= (A.n + 63) // 64
    if amg.num_levels() > 2:
        assert amg.stencil_layout_check(1) == (0, 0)


@pytest.mark.parametrize("gen,dims", [("7", (30, 27, 25)), ("7", (200, 180, 3)), ("27", (13, 12, 15)),
                                      ("aniso", (28, 26, 24))])
def test_coded_layout_rebuilds_rows(hv, gen, dims):
    """Offset-coded P_0 / R_0: every row decoded from its 16-bit codes (offset
    from the row's grid point, value index; P through the fine -> coarse map)
    equals the CSR row entry for entry, values bit for bit.  The 7-point
    hierarchy codes with the 25 offsets within distance 2; operators whose
    weights do not fit (the 27-point P_0: ~10^5 distinct values) report (0, 0)
    and keep the other layouts."""
    if gen == "27":
        A = hv.ParCSRMatrix.laplacian27(*dims)
    elif gen == "aniso":
        A = hv.ParCSRMatrix.laplacian(*dims, cx=0.001, cy=1.0, cz=1.0)
    else:
        A = hv.ParCSRMatrix.laplacian(*dims)
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=18)
    amg = hv.BoomerAMG(**kw)
    amg.setup_host(A)
    for which in (1, 2):
        no, nv = amg.coded_layout_check(0, which)
        if gen == "7":
            assert 1 <= no <= 25 and 1 <= nv <= 2048, (which, no, nv)
        else:
            assert (no, nv) == (0, 0) or (no >= 1 and nv >= 1)


@pytest.mark.parametrize("forward", [True, False])
def test_gs_packed_schedule_size(hv, forward):
    """BoomerAMG's default smoother at the north-star grid width: 4096-row
    blocks of a 512-wide 7-point grid are 8 x-lines with 519 dependency levels
    of at most 8 rows; the packed schedule sweeps 8 such blocks per wavefront,
    so it stores at most 1.3x the operator's entries (the one-level-per-slice
    layout it replaced padded every level to 64 lanes: about 8x) and needs about
    one step per level of a block."""
    A = hv.ParCSRMatrix.laplacian(512, 16, 8)
    amg = hv.BoomerAMG(**hv.ij_amg_defaults(0))
    amg.set(max_levels=1, relax_type=13)
    amg.setup_host(A)
    nb = 512 * 16 * 8 // 4096
    st = amg.gs_schedule_stats(0, forward, nb)
    assert st["entries"] <= 1.3 * st["nnz"], st
    assert st["teams"] == nb // 8, st
    assert st["max_steps"] <= 520, st
    amg.gs_schedule_check(nb)


def test_gs_self_check_models_the_kernel_fences(hv):
    """gs_schedule_self_check emulates the sweeps' U publication: a batch of
    kGsBatch = 4 steps is stored at its last step and fenced at the next
    batch's last step, and the pipelined sweep gathers step j's U values
    during step j - 1, so they must have been fenced by the end of step j - 2:
    a value is readable 9 steps after it was computed at the latest.  A
    schedule whose U codes reach back only 8 steps (knob 11 = 8 shortens the
    ring reach from 15 to 7) reads one step early and is refused."""
    A = hv.ParCSRMatrix.laplacian(14, 12, 11)
    amg = hv.BoomerAMG(**hv.ij_amg_defaults(0))
    amg.set(coarsen_type=8, relax_type=13, P_max_elmts=4)
    amg.setup_host(A)
    amg.gs_schedule_check(1)
    hv.set_knob(11, 6)  # U from 10 steps back: still published in time
    try:
        amg.gs_schedule_check(1)
    finally:
        hv.set_knob(11, 0)
    hv.set_knob(11, 8)
    try:
        with pytest.raises(Exception, match="differs from the sequential sweep"):
            amg.gs_schedule_check(1)
    finally:
        hv.set_knob(11, 0)
    amg.gs_schedule_check(1)


@pytest.mark.parametrize("nb", [1, 7])
def test_gs_schedule_16_lane_ring(hv, nb):
    """Knob 14 = 16: the small teams (team_rows 3 in the check) are cut into
    steps of at most 16 rows with 16-lane ring slots (ring codes slot x 16 +
    lane); every level, both directions, both scalings and the weighted form
    still equal the sequential sweep bit for bit, and every step starts on an
    even entry (the paired loads)."""
    A = hv.ParCSRMatrix.laplacian(14, 12, 11)
    amg = hv.BoomerAMG(**hv.ij_amg_defaults(0))
    amg.set(coarsen_type=8, relax_type=13, P_max_elmts=4)
    amg.setup_host(A)
    hv.set_knob(14, 16)
    try:
        amg.gs_schedule_check(nb)
    finally:
        hv.set_knob(14, 0)


@pytest.mark.parametrize("size", [2, 3, 5, 8])
@pytest.mark.parametrize("stencil,relax,interp,agg", [(7, 18, 6, 0), (27, 13, 6, 0), (7, 13, 14, 0), (7, 18, 6, 1),
                                                      (7, 18, 14, 2)])
def test_distributed_hmis_matches_rank_coarsening(hv, size, stencil, relax, interp, agg):
    """HMIS (coarsen_type 10, hypre's default) and extended interpolation (14)
    in the distributed setup: each rank's Ruge first pass over the strong
    connections it owns, then PMIS seeded with its C points with one random
    stream per rank (par_coarsen.c:2774 on N processes; dsetup.cpp hmis_dist).
    Every rank's part of every level equals the rank emulation's hierarchy
    byte for byte, with aggressive levels (the second pass per rank too)."""
    if stencil == 27:
        A = hv.ParCSRMatrix.laplacian27(17, 15, 19)
    else:
        A = hv.ParCSRMatrix.laplacian(19, 17, 23, cx=1.0 if agg == 0 else 0.3)
    amg = hv.BoomerAMG(**hv.ij_amg_defaults(0))
    amg.set(coarsen_type=10, interp_type=interp, relax_type=relax, P_max_elmts=4, agg_num_levels=agg)
    amg.dist_setup_check(A, size)


def test_hmis_rank_coarsening_has_teeth(hv):
    """The per-rank HMIS differs from the one-process HMIS (first pass over the
    whole graph), so the checks above compare against another hierarchy than
    the one-process setup's."""
    A = hv.ParCSRMatrix.laplacian(19, 17, 23)
    sizes = []
    for starts in (None, [0, A.n // 3, 2 * A.n // 3, A.n]):
        amg = hv.BoomerAMG(**hv.ij_amg_defaults(0))
        amg.set(coarsen_type=10, interp_type=6, relax_type=18, P_max_elmts=4)
        amg.set_coarsen_rank_starts(starts)
        amg.setup_host(A)
        sizes.append([amg.level_matrix(l, 0)[3][0] for l in range(amg.num_levels())])
        cf = amg.level_vector(0, 0)
        sizes[-1].append(cf.tobytes())
        amg.destroy()
    assert sizes[0] != sizes[1]


@pytest.mark.parametrize("coarsen,interp,agg,agg_interp", [(8, 16, 0, 4), (8, 17, 0, 4), (10, 18, 0, 4),
                                                            (8, 6, 1, 5), (8, 6, 1, 7), (10, 6, 1, 1), (8, 3, 0, 4)])
def test_distributed_setup_refuses_to_the_gathered_emulation(hv, coarsen, interp, agg, agg_interp):
    """The matrix-matrix interpolations (16-18), the 2-stage aggressive ones
    and the direct one (3) are not set up distributed: their products follow
    hypre_ParMatmul's N-rank entry order, which the rank emulation restates in
    one process, so an N-rank setup gathers the matrix on rank 0 and runs that
    emulation there (capi.hip setup_multi, GetSetupPath 3; the direct
    interpolation, which the emulation does not restate, path 4).  The
    distributed setup refuses them and says why."""
    A = hv.ParCSRMatrix.laplacian(11, 10, 12)
    amg = hv.BoomerAMG(**hv.ij_amg_defaults(0))
    amg.set(coarsen_type=coarsen, interp_type=interp, relax_type=18, P_max_elmts=4, agg_num_levels=agg,
            agg_interp_type=agg_interp)
    with pytest.raises(hv.HypreError, match="distributed setup: (interp_type|aggressive)"):
        amg.dist_setup_check(A, 2)


@pytest.mark.parametrize("size", [2, 3, 5, 8])
@pytest.mark.parametrize("coarsen,order,scale,variant,eig", [(8, 2, 1, 0, 10), (8, 3, 0, 1, 10), (10, 2, 1, 0, 10),
                                                             (8, 2, 1, 0, 0)])
def test_distributed_chebyshev_matches_one_process(hv, size, coarsen, order, scale, variant, eig):
    """Chebyshev (relax 16) in the distributed setup: the eigenvalue estimate's
    CG (par_relax_more.c:115) draws its start vector from every rank's own
    stream (seed my_id + 1, par_vector.c:337), and every inner product is a
    running sum handed from rank to rank in rank order, so the coefficients
    and the scaling equal the rank emulation's byte for byte; eig 0: the
    inf-norm bound (par_relax_more.c:25)."""
    A = hv.ParCSRMatrix.laplacian(19, 17, 23, cx=1.0, cy=0.5, cz=1.0)
    amg = hv.BoomerAMG(**hv.ij_amg_defaults(0))
    amg.set(coarsen_type=coarsen, interp_type=6, relax_type=16, P_max_elmts=4, cheby_order=order,
            cheby_scale=scale, cheby_variant=variant, cheby_eig_est=eig)
    amg.dist_setup_check(A, size)


@pytest.mark.parametrize("relax", [0, 18])
def test_scaled_norm_relax_weight(hv, relax):
    """relax_wt 0 (par_amg_setup.c:3184): every level's weight is 4/3 over
    max_i sum_j |a_ij| / sqrt(|a_ii|) / sqrt(|a_jj|) (par_scaled_matnorm.c:21,
    each row summed in stored order), recomputed here entry by entry."""
    A = hv.ParCSRMatrix.laplacian(14, 12, 10, cx=0.3)
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=8, relax_type=relax, relax_wt=0.0)
    amg = hv.BoomerAMG(**kw)
    amg.setup_host(A)
    for l in range(amg.num_levels()):
        ip, jj, vv, (nr, _) = amg.level_matrix(l, 0)
        ip, jj, vv = np.asarray(ip), np.asarray(jj), np.asarray(vv)
        dis = 1.0 / np.sqrt(np.abs(vv[ip[:-1]]))
        mx = 0.0
        for i in range(nr):
            s = 0.0
            for q in range(ip[i], ip[i + 1]):
                s += abs(vv[q]) * dis[i] * dis[jj[q]]
            mx = max(mx, s)
        w, _ = amg.level_weights(l)
        assert w == 4.0 / 3.0 / mx
    amg.destroy()
    A.destroy()


def test_dof_func_matches_interleaved_default(hv):
    """HYPRE_BoomerAMGSetDofFunc with the interleaved map (0, 1, 2, 0, ...) gives
    the hierarchy num_functions alone builds, and another partition of the rows
    into functions another one."""
    import scipy.sparse as sp  # noqa: F401
    sys.path.insert(0, os.path.join(os.path.dirname(__file__)))
    import ij_emul
    A_s, _ = ij_emul.sys_laplacian_ranks(8, 7, 6, 1, 1, 1, nf=3)
    A = hv.ParCSRMatrix.from_scipy(A_s)
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=8, num_functions=3)
    digests = []
    for dof in (None, [i % 3 for i in range(A.n)], [(i // 3) % 3 for i in range(A.n)]):
        amg = hv.BoomerAMG(**kw)
        amg.set_dof_func(dof)
        amg.setup_host(A)
        h = hashlib.sha256()
        for l in range(amg.num_levels()):
            ip, jj, vv, _ = amg.level_matrix(l, 0)
            h.update(np.asarray(jj).tobytes())
            h.update(np.asarray(vv).tobytes())
        digests.append(h.hexdigest())
        amg.destroy()
    assert digests[0] == digests[1]
    assert digests[0] != digests[2]
    A.destroy()
