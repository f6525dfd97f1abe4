"""Automatic hybrid Gauss-Seidel blocks (hypreve_BoomerAMGSetNumBlocks(0), the
default): level 0 gets one block per about 4096 rows, and that count (hypre's
thread count) is used on every level, capped so that a coarse level keeps
blocks of at least 64 rows instead of blocks of 0-1 rows (which would turn
relax 3/4/6 into unweighted Jacobi and relax 8/13/14 into l1-Jacobi).

CPU: the exported blocks and the convergence of relax 3 / 6 / 13 through the
oracle.  GPU: the same hierarchies, iterates bitwise equal to the oracle.
"""
import numpy as np
import pytest

AUTO = 4096
MIN_ROWS = 64


def amg_auto(hv, relax, **extra):
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=8, relax_type=relax, tol=1e-8, max_iter=60)
    kw.update(extra)
    return hv.BoomerAMG(**kw)  # num_blocks left at its default: automatic


@pytest.mark.parametrize("relax", [3, 6, 13])
def test_auto_blocks_per_level(hv, orc, relax):
    A = hv.ParCSRMatrix.laplacian(40, 36, 32)  # 46080 rows: 12 level-0 blocks
    amg = amg_auto(hv, relax)
    amg.setup_host(A)
    nl = amg.num_levels()
    assert nl >= 4
    top = -(-A.n // AUTO)
    for l in range(nl):
        n = amg.level_info(l)[0]
        bs = amg.level_vector(l, 3)
        nb = max(1, min(top, -(-n // MIN_ROWS)))
        assert bs.size == nb + 1, (l, n, bs.size)
        assert bs[0] == 0 and bs[-1] == n
        assert np.all(np.diff(bs) >= 1)
    # level 0 has several blocks, the small coarse levels blocks of >= 64 rows
    assert amg.level_vector(0, 3).size - 1 == 12
    assert amg.level_vector(1, 3).size - 1 == 12
    assert np.all(np.diff(amg.level_vector(nl - 2, 3)) >= MIN_ROWS) or amg.level_vector(nl - 2, 3).size == 2
    O = orc.OracleAMG(amg)
    st = O.solve(np.ones(A.n), np.zeros(A.n), 1e-8, 60)
    assert st["rel_res"] < 1e-8 and st["iterations"] <= 25, st
    amg.destroy()
    A.destroy()


def test_fixed_blocks_everywhere(hv):
    """num_blocks >= 1: that count on every level (hypre's OMP_NUM_THREADS)."""
    A = hv.ParCSRMatrix.laplacian(20, 20, 20)
    amg = amg_auto(hv, 6, num_blocks=3)
    amg.setup_host(A)
    assert amg.relax_info()["num_blocks"] == 3
    for l in range(amg.num_levels()):
        assert amg.level_vector(l, 3).size == 0  # the num_blocks partition (no per-level export)
    amg.destroy()
    A.destroy()


@pytest.mark.gpu
@pytest.mark.parametrize("relax", [3, 6, 13])
def test_gpu_auto_blocks_bitwise(gpu, orc, relax):
    hv = gpu
    A = hv.ParCSRMatrix.laplacian(40, 36, 32)
    amg = amg_auto(hv, relax)
    amg.setup(A)
    n = A.n
    b = hv.ParVector(n, np.ones(n))
    x = hv.ParVector(n, np.zeros(n))
    it, rr = amg.solve(A, b, x)
    u = np.zeros(n)
    st = orc.OracleAMG(amg).solve(np.ones(n), u, 1e-8, 60)
    assert it == st["iterations"] and rr < 1e-8
    assert np.array_equal(x.get(), u)
    amg.destroy()
    A.destroy()
