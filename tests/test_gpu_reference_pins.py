"""GPU solve path on the reference's np > 1 runs (tests/golden/ij_rank_fixtures.json).

HYPRE_BoomerAMGSetup with hypreve_BoomerAMGSetRankEmulation builds the
hierarchy an N-rank reference run builds, and the HIP cycle runs it with one
hybrid-GS block per rank.  Stand-alone BoomerAMG: the GPU iterate equals the
oracle's bit for bit and the printed statistics equal the saved ones (this is
where the weighted l1 hybrid GS of smoother.out.0, w = 1.1, and the C/F-ordered
relax 0 / 18 / 13-14 runs meet the reference's numbers on the GPU).  PCG: the
saved iteration count and the saved final relative residual to its printed
digits (PCG's dot products reduce in another order than the oracle's; 1e-6
relative).
"""
import numpy as np
import pytest

from test_reference_pins import CASES, build, check_stats, initial_guess

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_gpu_rank_fixture(gpu, orc, case):
    hv = gpu
    A, amg, b_h, starts = build(hv, case)
    n = A.n
    b = hv.ParVector(n, b_h)
    x0 = initial_guess(case, starts, n)
    x = hv.ParVector(n, x0)
    if case["solver"] == "amg":
        amg.setup(A)
        it, rr = amg.solve(A, b, x)
        O = orc.OracleAMG(amg)
        u = x0.copy()
        st = O.solve(b_h, u, 1e-8, 100)
        assert it == st["iterations"]
        assert np.array_equal(x.get(), u), "GPU iterate differs from the oracle"
        assert abs(rr - st["rel_res"]) <= 1e-10 * st["rel_res"]
        check_stats(case, amg, st, it, st["rel_res"])
    else:
        pcg = hv.PCG(tol=1e-8, max_iter=1000, two_norm=1)
        pcg.set_precond_amg(amg)
        pcg.setup(A, b, x)
        it, rr = pcg.solve(A, b, x)
        exp = case["expect"]
        assert it == exp["iterations"]
        assert abs(rr - exp["rel_res"]) <= 1e-6 * exp["rel_res"] + 5e-16
        pcg.destroy()
    amg.destroy()
    A.destroy()


@pytest.mark.parametrize("relax,nb", [(3, 1), (6, 3), (13, 2), (14, 1), (8, 4), (4, 2)])
@pytest.mark.parametrize("w,omega", [(1.1, 1.0), (0.8, 1.3), (1.0, 0.7)])
def test_gpu_weighted_hybrid_gs_bitwise(gpu, orc, relax, nb, w, omega):
    """Weighted hybrid GS / SOR (relax_weight, outer weight != 1; par_relax.c
    :1277, :2075, :3150, :3785, :4544, :4937) on the GPU equals the oracle bit
    for bit, one V-cycle and a solve, on thread blocks and a level-0 weight."""
    hv = gpu
    A = hv.ParCSRMatrix.laplacian(21, 19, 17)
    kw = hv.ij_amg_defaults(0)
    kw.update(relax_type=relax, num_blocks=nb, relax_wt=w, outer_wt=omega, max_iter=6, tol=0.0)
    amg = hv.BoomerAMG(**kw)
    amg.set(level_relax_wt=(1.05, 0))
    amg.setup(A)
    n = A.n
    rng = np.random.default_rng(3)
    f_h = rng.standard_normal(n)
    u0 = rng.standard_normal(n)
    f = hv.ParVector(n, f_h)
    u = hv.ParVector(n, u0)
    amg.cycle(f, u)
    O = orc.OracleAMG(amg)
    uo = u0.copy()
    O.cycle(f_h, uo)
    assert np.array_equal(u.get(), uo)
    x = hv.ParVector(n, np.zeros(n))
    amg.solve(A, f, x)
    xo = np.zeros(n)
    O.solve(f_h, xo, 0.0, 6)
    assert np.array_equal(x.get(), xo)
    # the weights change the iterate (the test has teeth)
    amg2 = hv.BoomerAMG(**dict(kw, relax_wt=1.0, outer_wt=1.0))
    amg2.setup(A)
    O2 = orc.OracleAMG(amg2)
    u2 = u0.copy()
    O2.cycle(f_h, u2)
    assert not np.array_equal(u2, uo)
