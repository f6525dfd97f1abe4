"""GPU parity: the HIP solve path (through the C ABI) against the CPU oracle.

Stand-alone BoomerAMG iterates involve no reductions, and every device kernel
forms each row sum in the reference's order without FMA contraction, so the
GPU iterate must equal the oracle's bit for bit (np.array_equal, +0 == -0).
Residual norms and PCG scalars involve reductions in a different order; they
are compared with a stated tolerance (rtol 1e-10 on relative residuals).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RTOL_NORM = 1e-10


def setup_pair(hv, orc, n3, **settings):
    A = hv.ParCSRMatrix.laplacian(*n3)
    kw = hv.ij_amg_defaults(0)
    kw.update(settings)
    amg = hv.BoomerAMG(**kw)
    amg.setup(A)
    return A, amg, orc.OracleAMG(amg)


@pytest.mark.parametrize("relax", [0, 18])
def test_fixture_default_on_gpu(gpu, orc, relax):
    """default.out.0 (TEST_ij/default.saved) solved on the GPU: same iterates."""
    hv = gpu
    A, amg, O = setup_pair(hv, orc, (10, 10, 10), coarsen_type=8, P_max_elmts=0, relax_type=relax)
    n = A.n
    b_h = O.matvec(0, 1.0, np.ones(n), 0.0, np.zeros(n))
    b = hv.ParVector(n, b_h)
    x = hv.ParVector(n, np.zeros(n))
    it, rr = amg.solve(A, b, x)
    u = np.zeros(n)
    st = O.solve(b_h, u, 1e-8, 100)
    assert it == st["iterations"]
    assert np.array_equal(x.get(), u)
    assert abs(rr - st["rel_res"]) <= RTOL_NORM * st["rel_res"]
    if relax == 0:
        assert it == 48


@pytest.mark.parametrize("n3,relax,coarsen", [((24, 20, 16), 18, 8), ((17, 13, 11), 0, 8), ((33, 33, 33), 18, 8),
                                              ((24, 20, 16), 18, 10), ((31, 29, 27), 0, 10), ((23, 19, 17), 18, 11),
                                              ((22, 18, 15), 17, 8)])
def test_single_cycle_bitwise(gpu, orc, n3, relax, coarsen):
    """One V-cycle from a random iterate; coarsen 10 = HMIS (test/ij.c default),
    11 = the Ruge first pass alone (ij -ruge1p); relax 17 = FCF-Jacobi."""
    hv = gpu
    A, amg, O = setup_pair(hv, orc, n3, coarsen_type=coarsen, relax_type=relax)
    n = A.n
    rng = np.random.default_rng(7)
    f_h = rng.standard_normal(n)
    u0 = rng.standard_normal(n)
    f = hv.ParVector(n, f_h)
    u = hv.ParVector(n, u0)
    amg.cycle(f, u)
    uo = u0.copy()
    O.cycle(f_h, uo)
    assert np.array_equal(u.get(), uo)


@pytest.mark.parametrize("relax,coarsen,wt", [(18, 8, 1.0), (0, 8, 1.0), (18, 10, 1.0), (7, 10, 1.0),
                                              (18, 8, 0.8), (7, 8, 1.0), (0, 8, 0.0), (18, 10, 0.0)])
def test_cf_relaxation_cycle_bitwise(gpu, orc, relax, coarsen, wt):
    """relax_order 1 (C points, then F points on the way down; F then C up).
    relax 18: hypre_ParCSRRelax_L1_Jacobi per point class with the C/F-restricted
    l1 norms (par_cycle.c:398-415, par_relax_more.c:991); relax 7: two full
    sweeps (RelaxIF, par_relax.c:3463 ignores relax_points); relax 0: C/F Jacobi.
    wt 0: every level's weight is 4/3 over its scaled norm (par_amg_setup.c:3184).
    The oracle's C/F sweep is itself checked against the formula in
    tests/test_oracle_relax.py.  Control: the same hierarchy with relax_order 0
    gives different bits, so the C/F path is really taken."""
    hv = gpu
    A, amg, O = setup_pair(hv, orc, (26, 22, 19), coarsen_type=coarsen, relax_type=relax, relax_order=1,
                           relax_wt=wt)
    n = A.n
    rng = np.random.default_rng(17)
    f_h = rng.standard_normal(n)
    u0 = rng.standard_normal(n)
    f = hv.ParVector(n, f_h)
    u = hv.ParVector(n, u0)
    amg.cycle(f, u)
    uo = u0.copy()
    O.cycle(f_h, uo)
    assert np.array_equal(u.get(), uo)
    O.s.relax_order = 0
    uc = u0.copy()
    O.cycle(f_h, uc)
    assert not np.array_equal(uc, uo)
    # a solve with the fused solve-loop kernels switched off by relax_order 1
    b = hv.ParVector(n, f_h)
    x = hv.ParVector(n, np.zeros(n))
    amg.set(tol=1e-7, max_iter=30)
    it, rr = amg.solve(A, b, x)
    O.s.relax_order = 1
    xo = np.zeros(n)
    st = O.solve(f_h, xo, 1e-7, 30)
    assert it == st["iterations"]
    assert np.array_equal(x.get(), xo)


@pytest.mark.parametrize("policy", [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15])
@pytest.mark.parametrize("relax,order", [(18, 0), (0, 1)])
def test_sell_policy_cycle_bitwise(gpu, orc, policy, relax, order):
    """Every device layout / row loop (padded lane-per-row, jagged lane-per-row,
    workgroup-per-slice, jagged wave-product-parallel, jagged with an LDS
    x-tile, padded with 16-bit column deltas, the same with a value table,
    padded / jagged with 16-bit value indices, the slot-uniform stencil
    layout where an operator is a constant-coefficient stencil, offset-coded P
    and R where they build, packed 32-bit P and R codes) forced on every
    operator of the hierarchy: the same bits as the oracle.  The automatic
    choice only uses jagged and wide loops on operators too large for the
    other tests, so this is where those loops meet the oracle."""
    hv = gpu
    A, amg, O = setup_pair(hv, orc, (30, 27, 25), coarsen_type=8, interp_type=6, P_max_elmts=4,
                           relax_type=relax, relax_order=order, sell_policy=policy)
    n = A.n
    if policy == 12:  # the layout is really taken (level 0's P and R)
        assert amg.level_layout(0, 1) == "coded" and amg.level_layout(0, 2) == "coded"
    if policy == 15:  # R in the jagged, product-parallel coded form (k_code_pw), P padded
        assert amg.level_layout(0, 1) == "coded" and amg.level_layout(0, 2) == "coded-jag"
    if policy == 13:
        assert amg.level_layout(0, 1) == "packed" and amg.level_layout(0, 2) == "packed"
    if policy == 5:  # the lane-packed dictionary streams (k_sell_dictw), A's 4-slice groups included
        assert amg.level_layout(0, 0) == "dict-wide" and amg.level_layout(1, 0) == "dict-wide"
    if policy == 14:  # the per-entry dictionary streams (k_sell_dict)
        assert amg.level_layout(0, 0) == "dict" and amg.level_layout(1, 0) == "dict"
    rng = np.random.default_rng(23 + policy)
    f_h = rng.standard_normal(n)
    u0 = rng.standard_normal(n)
    f = hv.ParVector(n, f_h)
    u = hv.ParVector(n, u0)
    amg.cycle(f, u)
    uo = u0.copy()
    O.cycle(f_h, uo)
    assert np.array_equal(u.get(), uo)
    b = hv.ParVector(n, f_h)
    x = hv.ParVector(n, np.zeros(n))
    amg.set(tol=1e-7, max_iter=40)
    it, rr = amg.solve(A, b, x)
    xo = np.zeros(n)
    st = O.solve(f_h, xo, 1e-7, 40)
    assert it == st["iterations"]
    assert np.array_equal(x.get(), xo)


@pytest.mark.parametrize("kc,nopf", [(4, 0), (8, 1), (16, 0)])
def test_code_pw_chunk_variants_bitwise(gpu, orc, kc, nopf):
    """The jagged coded loop's launch variants (knob 4: entries per row and
    chunk, knob 5: no code prefetch) give the same bits: R_0 and the cycle."""
    hv = gpu
    A, amg, O = setup_pair(hv, orc, (30, 27, 25), coarsen_type=8, interp_type=6, P_max_elmts=4,
                           relax_type=18, sell_policy=15)
    assert amg.level_layout(0, 2) == "coded-jag"
    n = A.n
    rng = np.random.default_rng(5 + kc)
    f_h = rng.standard_normal(n)
    u0 = rng.standard_normal(n)
    f = hv.ParVector(n, f_h)
    u = hv.ParVector(n, u0)
    hv.set_knob(4, kc)
    hv.set_knob(5, nopf)
    try:
        amg.cycle(f, u)
    finally:
        hv.set_knob(4, 0)
        hv.set_knob(5, 0)
    uo = u0.copy()
    O.cycle(f_h, uo)
    assert np.array_equal(u.get(), uo)


@pytest.mark.parametrize("policy", [6, 7, 11])
def test_delta_layout_wide_stride_bitwise(gpu, orc, policy):
    """16-bit column deltas where the z-neighbour is 36000 rows away: the
    per-slot base carries the stride, and the z = 0 / z = last planes (one
    neighbour missing) put a padding slot between a row's entries.  One cycle
    and the residual equal the oracle's bits."""
    hv = gpu
    A, amg, O = setup_pair(hv, orc, (200, 180, 3), coarsen_type=8, interp_type=6, P_max_elmts=4,
                           relax_type=18, sell_policy=policy)
    n = A.n
    rng = np.random.default_rng(5)
    f_h = rng.standard_normal(n)
    u0 = rng.standard_normal(n)
    f = hv.ParVector(n, f_h)
    u = hv.ParVector(n, u0)
    if policy == 11:
        assert amg.level_layout(0, 0) == "stencil"
    amg.cycle(f, u)
    uo = u0.copy()
    O.cycle(f_h, uo)
    assert np.array_equal(u.get(), uo)


@pytest.mark.parametrize("coef", [(0.001, 1.0, 1.0), (1.0, 1.0, 100.0)])
def test_anisotropic_solve_bitwise(gpu, orc, coef):
    """configs[4]'s operator family at test size: anisotropic diffusion
    (GenerateLaplacian with cx, cy, cz), PMIS + ext+i Pmx 4, l1-Jacobi.  The
    strong-coupling pattern is one-dimensional, rows of the Galerkin levels are
    irregular; the GPU iterates equal the oracle's bit for bit."""
    hv = gpu
    A = hv.ParCSRMatrix.laplacian(28, 26, 24, cx=coef[0], cy=coef[1], cz=coef[2])
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=18, tol=1e-7, max_iter=60)
    amg = hv.BoomerAMG(**kw)
    amg.setup(A)
    O = orc.OracleAMG(amg)
    n = A.n
    rng = np.random.default_rng(31)
    b_h = rng.standard_normal(n)
    b = hv.ParVector(n, b_h)
    x = hv.ParVector(n, np.zeros(n))
    it, rr = amg.solve(A, b, x)
    xo = np.zeros(n)
    st = O.solve(b_h, xo, 1e-7, 60)
    assert it == st["iterations"]
    assert np.array_equal(x.get(), xo)


@pytest.mark.parametrize("order,scale,variant", [(2, 1, 0), (1, 1, 0), (3, 0, 0), (4, 1, 1), (2, 0, 1)])
def test_chebyshev_cycle_bitwise(gpu, orc, order, scale, variant):
    """Relax type 16 (par_cheby.c:166 scaled / unscaled Chebyshev, standard
    and modified polynomial): V-cycles and a solve equal the oracle's bits."""
    hv = gpu
    A, amg, O = setup_pair(hv, orc, (23, 21, 19), coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=16,
                           cheby_order=order, cheby_scale=scale, cheby_variant=variant)
    n = A.n
    rng = np.random.default_rng(41 + order)
    f_h = rng.standard_normal(n)
    u0 = rng.standard_normal(n)
    f = hv.ParVector(n, f_h)
    u = hv.ParVector(n, u0)
    amg.cycle(f, u)
    uo = u0.copy()
    O.cycle(f_h, uo)
    assert np.array_equal(u.get(), uo)
    b = hv.ParVector(n, f_h)
    x = hv.ParVector(n, np.zeros(n))
    amg.set(tol=1e-8, max_iter=40)
    it, rr = amg.solve(A, b, x)
    xo = np.zeros(n)
    st = O.solve(f_h, xo, 1e-8, 40)
    assert it == st["iterations"]
    assert np.array_equal(x.get(), xo)


def test_matvec_bitwise(gpu, orc):
    hv = gpu
    A, amg, O = setup_pair(hv, orc, (20, 20, 20), coarsen_type=8, relax_type=18)
    n = A.n
    rng = np.random.default_rng(3)
    xh, yh = rng.standard_normal(n), rng.standard_normal(n)
    for alpha, beta in [(1.0, 0.0), (-1.0, 1.0), (1.0, -1.0), (2.5, 0.5), (-0.7, 1.0)]:
        x, y = hv.ParVector(n, xh), hv.ParVector(n, yh)
        A.matvec(alpha, x, beta, y)
        ref = O.matvec(0, alpha, xh, beta, yh)
        assert np.array_equal(y.get(), ref), (alpha, beta)


def test_pcg_amg_l1jacobi(gpu, orc):
    """ij -solver 1 style: PCG (two-norm) + one BoomerAMG V-cycle (l1-Jacobi)."""
    hv = gpu
    A = hv.ParCSRMatrix.laplacian(32, 32, 32)
    amg = hv.BoomerAMG(**hv.ij_amg_defaults(1))
    amg.set(coarsen_type=8, relax_type=18)
    pcg = hv.PCG(tol=1e-8, max_iter=200, two_norm=1)
    pcg.set_precond_amg(amg)
    n = A.n
    rng = np.random.default_rng(11)
    b_h = rng.uniform(-1, 1, n)
    b = hv.ParVector(n, b_h)
    x = hv.ParVector(n, np.zeros(n))
    pcg.setup(A, b, x)
    it, rr = pcg.solve(A, b, x)
    O = orc.OracleAMG(amg)
    xo = np.zeros(n)
    ito, rro = O.pcg(b_h, xo, 1e-8, 200, 1)
    assert it == ito
    assert abs(rr - rro) <= 1e-6 * rro
    assert np.allclose(x.get(), xo, rtol=1e-9, atol=1e-12)
    assert rr < 1e-8


@pytest.mark.parametrize("relax", [None, 18])
def test_pcg_ij_64(gpu, orc, relax):
    """BASELINE configs[0]: ij's 3-D 7-point Laplacian 64^3, BoomerAMG-PCG
    (-solver 1), with ij's BoomerAMG settings (HMIS, ext+i Pmx 4, hybrid l1
    Gauss-Seidel 13/14 down/up, Gaussian elimination coarsest; relax=18: the
    l1-Jacobi variant the bench runs).  Same PCG iteration count as the CPU
    oracle and final relative residuals within 1e-6 (PCG's dot products are
    reduced in a different order)."""
    hv = gpu
    A = hv.ParCSRMatrix.laplacian(64, 64, 64)
    amg = hv.BoomerAMG(**hv.ij_amg_defaults(1))
    if relax is not None:
        amg.set(relax_type=relax)
    pcg = hv.PCG(tol=1e-8, max_iter=100, two_norm=1)
    pcg.set_precond_amg(amg)
    n = A.n
    b_h = np.ones(n)
    b = hv.ParVector(n, b_h)
    x = hv.ParVector(n, np.zeros(n))
    pcg.setup(A, b, x)
    it, rr = pcg.solve(A, b, x)
    O = orc.OracleAMG(amg)
    xo = np.zeros(n)
    ito, rro = O.pcg(b_h, xo, 1e-8, 100, 1)
    assert it == ito
    assert abs(rr - rro) <= 1e-6 * rro
    assert rr < 1e-8
    assert np.allclose(x.get(), xo, rtol=1e-9, atol=1e-12)


def test_large_solve_properties(gpu):
    """128^3 (2.1M rows): the GPU V-cycle converges monotonically and its
    average factor is in the range the reference reports for this stencil."""
    hv = gpu
    A = hv.ParCSRMatrix.laplacian(128, 128, 128)
    amg = hv.BoomerAMG(**hv.ij_amg_defaults(0))
    amg.set(coarsen_type=8, relax_type=18, tol=1e-8, max_iter=60)
    amg.setup(A)
    n = A.n
    b = hv.ParVector(n, np.ones(n))
    x = hv.ParVector(n, np.zeros(n))
    it, rr = amg.solve(A, b, x)
    assert rr < 1e-8
    assert it < 60
    # residual check via the GPU matvec: r = b - A x
    r = hv.ParVector(n, np.ones(n))
    A.matvec(-1.0, x, 1.0, r)
    assert np.sqrt(r.dot(r)) / np.sqrt(n) < 2e-8


@pytest.mark.parametrize("relax", [3, 4, 6, 8, 13, 14])
@pytest.mark.parametrize("num_blocks", [1, 13, 256])
def test_hybrid_gs_cycle_bitwise(gpu, orc, relax, num_blocks):
    """Hybrid Gauss-Seidel (par_relax.c cases 3/4/6/8/13/14) with num_blocks =
    hypre's thread blocks, run on the GPU as per-block level schedules: one
    V-cycle equals the oracle's sequential per-block sweeps bit for bit."""
    hv = gpu
    A, amg, O = setup_pair(hv, orc, (18, 14, 12), coarsen_type=8, relax_type=relax, num_blocks=num_blocks)
    n = A.n
    rng = np.random.default_rng(relax * 100 + num_blocks)
    f_h = rng.standard_normal(n)
    u0 = rng.standard_normal(n)
    f = hv.ParVector(n, f_h)
    u = hv.ParVector(n, u0)
    amg.cycle(f, u)
    uo = u0.copy()
    O.cycle(f_h, uo)
    assert np.array_equal(u.get(), uo)


@pytest.mark.parametrize("coarsen", [8, 10])
def test_boomeramg_default_smoothers_solve(gpu, orc, coarsen):
    """BoomerAMG's default smoothers (l1 hybrid GS forward down, backward up,
    Gaussian elimination coarsest: relax 13 / 14 / 9) over a whole solve."""
    hv = gpu
    A, amg, O = setup_pair(hv, orc, (20, 20, 20), coarsen_type=coarsen, num_blocks=64,
                           cycle_relax_type={1: 13, 2: 14, 3: 9})
    n = A.n
    b = hv.ParVector(n, np.ones(n))
    x = hv.ParVector(n, np.zeros(n))
    it, rr = amg.solve(A, b, x)
    u = np.zeros(n)
    st = O.solve(np.ones(n), u, 1e-8, 100)
    assert it == st["iterations"]
    assert np.array_equal(x.get(), u)
    assert abs(rr - st["rel_res"]) <= RTOL_NORM * st["rel_res"]


@pytest.mark.parametrize("agg,coarsen,relax", [(1, 8, 18), (2, 8, 18), (1, 10, 18), (1, 8, 13), (10, 10, 6)])
@pytest.mark.parametrize("coef", [(0.001, 1.0, 1.0), (1.0, 1.0, 1.0)])
def test_aggressive_coarsening_bitwise(gpu, orc, agg, coarsen, relax, coef):
    """configs[4]: anisotropic diffusion with PMIS / HMIS and aggressive levels
    (second coarsening on S*S + 2S, multipass interpolation; par_amg_setup.c
    :1239-1285, par_multi_interp.c:16).  The irregular rows of the aggressive
    Galerkin levels run through the automatic layouts; one V-cycle and a solve
    equal the oracle's bits."""
    hv = gpu
    A = hv.ParCSRMatrix.laplacian(28, 26, 24, cx=coef[0], cy=coef[1], cz=coef[2])
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=coarsen, agg_num_levels=agg, relax_type=relax, num_blocks=16, tol=1e-7, max_iter=80)
    amg = hv.BoomerAMG(**kw)
    amg.setup(A)
    O = orc.OracleAMG(amg)
    n = A.n
    rng = np.random.default_rng(agg * 10 + coarsen)
    f_h = rng.standard_normal(n)
    u0 = rng.standard_normal(n)
    f = hv.ParVector(n, f_h)
    u = hv.ParVector(n, u0)
    amg.cycle(f, u)
    uo = u0.copy()
    O.cycle(f_h, uo)
    assert np.array_equal(u.get(), uo)
    b = hv.ParVector(n, f_h)
    x = hv.ParVector(n, np.zeros(n))
    it, rr = amg.solve(A, b, x)
    xo = np.zeros(n)
    st = O.solve(f_h, xo, 1e-7, 80)
    assert it == st["iterations"]
    assert np.array_equal(x.get(), xo)


@pytest.mark.parametrize("interp,agg,agg_interp", [(14, 0, 4), (16, 0, 4), (17, 0, 4), (18, 0, 4), (6, 1, 5), (6, 2, 5), (18, 1, 5), (6, 1, 7),
                                                     (6, 1, 1), (6, 2, 3), (6, 1, 6), (8, 0, 4), (6, 1, 2),
                                                     (7, 0, 4)])
@pytest.mark.parametrize("order", [0, 1])
def test_interp_types_bitwise(gpu, orc, interp, agg, agg_interp, order):
    """Extended (14), ext / ext+i / ext+e MM (16 / 17 / 18) and the 2-stage extended / ext+e MM
    aggressive interpolations (agg_interp_type 5 / 7, whose levels keep -2
    markers that C/F relaxation skips), and the classical 2-stage ext+i / ext
    and MM ext+i ones (agg_interp_type 1 / 3 / 6, partial.c), standard
    interpolation (8) and its 2-stage form (agg_interp_type 2): one V-cycle and
    a solve equal the oracle's bits."""
    hv = gpu
    A = hv.ParCSRMatrix.laplacian(28, 26, 24, cx=0.01)
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=8, interp_type=interp, agg_num_levels=agg, agg_interp_type=agg_interp,
              relax_type=18, relax_order=order, tol=1e-7, max_iter=80)
    amg = hv.BoomerAMG(**kw)
    amg.setup(A)
    O = orc.OracleAMG(amg)
    n = A.n
    rng = np.random.default_rng(interp * 7 + agg)
    f_h = rng.standard_normal(n)
    u0 = rng.standard_normal(n)
    f = hv.ParVector(n, f_h)
    u = hv.ParVector(n, u0)
    amg.cycle(f, u)
    uo = u0.copy()
    O.cycle(f_h, uo)
    assert np.array_equal(u.get(), uo)
    b = hv.ParVector(n, f_h)
    x = hv.ParVector(n, np.zeros(n))
    it, rr = amg.solve(A, b, x)
    xo = np.zeros(n)
    st = O.solve(f_h, xo, 1e-7, 80)
    assert it == st["iterations"]
    assert np.array_equal(x.get(), xo)


# grids with 64 | nx and from 2^18 rows up (the stencil layout); ny and nz not
# multiples of the tile (16 lines) or of the planes a workgroup marches
@pytest.mark.parametrize("gen,n3,relax,wt,zc", [("7", (64, 64, 64), 18, 1.0, 0), ("27", (64, 66, 64), 18, 1.0, 7),
                                                ("aniso", (128, 40, 52), 18, 1.0, 0), ("7", (192, 50, 30), 18, 0.8, 5),
                                                ("27", (128, 37, 60), 0, 1.0, 0), ("7", (64, 64, 70), 13, 1.0, 64)])
def test_grid_stencil_bitwise(gpu, orc, gen, n3, relax, wt, zc):
    """The grid-stencil loop (k_grid_stencil: x staged in an LDS ring of tile
    planes) on level 0: a V-cycle from a random iterate and a 3-iteration
    solve (the fused residual + first sweep, its norm) equal the oracle bit
    for bit with l1-Jacobi (weight 1 and 0.8), Jacobi and hybrid GS, and the
    layout is really the grid form.  zc: planes a workgroup marches (knob 9;
    0 = automatic)."""
    hv = gpu
    if gen == "27":
        A = hv.ParCSRMatrix.laplacian27(*n3)
    elif gen == "aniso":
        A = hv.ParCSRMatrix.laplacian(*n3, cx=0.001, cy=1.0, cz=1.0)
    else:
        A = hv.ParCSRMatrix.laplacian(*n3)
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=8, relax_type=relax, relax_wt=wt, P_max_elmts=4)
    amg = hv.BoomerAMG(**kw)
    hv.set_knob(9, zc)
    try:
        amg.setup(A)
    finally:
        hv.set_knob(9, 0)
    assert amg.level_layout(0, 0) == "grid-stencil"
    O = orc.OracleAMG(amg)
    n = A.n
    rng = np.random.default_rng(29)
    f_h = rng.standard_normal(n)
    u0 = rng.standard_normal(n)
    f = hv.ParVector(n, f_h)
    u = hv.ParVector(n, u0)
    amg.cycle(f, u)
    uo = u0.copy()
    O.cycle(f_h, uo)
    assert np.array_equal(u.get(), uo)
    amg.set(tol=0.0, max_iter=3)
    x = hv.ParVector(n, np.zeros(n))
    it, rr = amg.solve(A, f, x)
    xo = np.zeros(n)
    st = O.solve(f_h, xo, 0.0, 3)
    assert np.array_equal(x.get(), xo)
    assert abs(rr - st["rel_res"]) <= RTOL_NORM * st["rel_res"]
    for alpha, beta in [(1.0, 0.0), (-1.0, 1.0), (2.5, 0.5)]:
        xv, yv = hv.ParVector(n, u0), hv.ParVector(n, f_h)
        A.matvec(alpha, xv, beta, yv)
        assert np.array_equal(yv.get(), O.matvec(0, alpha, u0, beta, f_h)), (alpha, beta)


def test_grid_stencil_thin_grid_norm_parts(gpu, orc):
    """A thin grid (ny = 3: one line of tiles, every tile mostly empty lines)
    on the grid-stencil loop gives far more per-wave norm partials (2048 tiles
    x 8 waves) than rows / 64: the fused residual + first sweep with its norm
    and the PCG matvec-dot must fit the workspace (DevAMG::size_nrm_parts) and
    equal the oracle (solve: bitwise; norms and PCG: rtol)."""
    hv = gpu
    A = hv.ParCSRMatrix.laplacian(64, 3, 4096)
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=8, relax_type=18, P_max_elmts=4)
    amg = hv.BoomerAMG(**kw)
    amg.setup(A)
    assert amg.level_layout(0, 0) == "grid-stencil"
    O = orc.OracleAMG(amg)
    n = A.n
    rng = np.random.default_rng(5)
    f_h = rng.standard_normal(n)
    f = hv.ParVector(n, f_h)
    amg.set(tol=0.0, max_iter=3)
    x = hv.ParVector(n, np.zeros(n))
    it, rr = amg.solve(A, f, x)
    xo = np.zeros(n)
    st = O.solve(f_h, xo, 0.0, 3)
    assert np.array_equal(x.get(), xo)
    assert abs(rr - st["rel_res"]) <= RTOL_NORM * st["rel_res"]
    # BoomerAMG-PCG on the same hierarchy: s = A p with <s, p> fused
    amg.set(tol=0.0, max_iter=1)
    kr = hv.PCG(tol=0.0, max_iter=4, two_norm=1)
    kr.set_precond_amg(amg, setup=False)
    kr.setup(A, f, x)
    x.fill(0.0)
    it_g, rr_g = kr.solve(A, f, x)
    kr.destroy()
    u = np.zeros(n)
    it_o, rr_o = O.pcg(f_h, u, 0.0, 4, 1)
    assert it_g == it_o == 4
    assert np.linalg.norm(x.get() - u) <= 1e-9 * np.linalg.norm(u)


@pytest.mark.parametrize("cycle_type,num_sweeps,relax", [(2, 1, 18), (2, 2, 18), (1, 2, 18), (2, 2, 13), (2, 1, 0)])
def test_w_cycle_sweeps_bitwise(gpu, orc, cycle_type, num_sweeps, relax):
    """cycle_type 2 (W-cycle: lev_counter, par_cycle.c:246-250 / :683-700) and
    num_sweeps 2 on every level but the coarsest: a cycle from a random
    iterate and a 4-iteration solve equal the oracle bit for bit, on a
    hierarchy deep enough (64^3 and 24^3 levels below) that the W-cycle's
    repeated coarse visits differ from the V-cycle (control below)."""
    hv = gpu
    A, amg, O = setup_pair(hv, orc, (48, 44, 40), coarsen_type=8, relax_type=relax, P_max_elmts=4,
                           cycle_type=cycle_type, num_sweeps=num_sweeps)
    info = amg.relax_info()
    assert info["cycle_type"] == cycle_type
    n = A.n
    rng = np.random.default_rng(41)
    f_h = rng.standard_normal(n)
    u0 = rng.standard_normal(n)
    f = hv.ParVector(n, f_h)
    u = hv.ParVector(n, u0)
    amg.cycle(f, u)
    uo = u0.copy()
    O.cycle(f_h, uo)
    assert np.array_equal(u.get(), uo)
    amg.set(tol=0.0, max_iter=4)
    x = hv.ParVector(n, np.zeros(n))
    amg.solve(A, f, x)
    xo = np.zeros(n)
    O.solve(f_h, xo, 0.0, 4)
    assert np.array_equal(x.get(), xo)
    if cycle_type == 2:
        O.s.cycle_type = 1
        uv = u0.copy()
        O.cycle(f_h, uv)
        assert not np.array_equal(uv, uo)
