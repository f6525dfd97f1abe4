"""The oracle's smoothers against hand-written numpy statements of the
reference formulas (CPU only).

* relax 18 with relax_points = +-1: hypre_ParCSRRelax_L1_Jacobi
  (par_relax_more.c:991-1152): Vtemp = u, then for every row i of the class
  with a nonzero diagonal, u_i += (w * (f_i - sum_j a_ij Vtemp_j)) / l1_i.
* relax 7 ignores relax_points (par_relax.c:3463): a C/F-ordered call through
  hypre_BoomerAMGRelaxIF is a full Jacobi sweep each time.
* relax 18 with relax_points = 0 (ams.c:41 hypre_ParCSRRelax type 1):
  v = w f - w A u (matvec -w, +w), u += v / l1.

Row sums run in stored order with every product rounded (no FMA), as the
oracle does, so the comparisons are bitwise.
"""
import ctypes as C

import numpy as np
import pytest


def diag_first_csr(n, seed, zero_diag_rows=()):
    rng = np.random.default_rng(seed)
    ip, jj, vv = [0], [], []
    for i in range(n):
        cols = sorted(set(rng.integers(0, n, size=5).tolist()) - {i})
        d = 0.0 if i in zero_diag_rows else 6.0 + rng.random()
        jj += [i] + cols
        vv += [d] + (-rng.random(len(cols))).tolist()
        ip.append(len(jj))
    return np.array(ip, np.int32), np.array(jj, np.int32), np.array(vv, np.float64)


def row_res(ip, jj, vv, f, x, i):
    r = f[i]
    for k in range(ip[i], ip[i + 1]):
        r = r - vv[k] * x[jj[k]]
    return r


def relax(orc, A, f, cf, rt, pts, w, l1, u):
    L = orc.lib()
    n = A.nrows
    vt, zt = np.zeros(n), np.zeros(n)
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))
    rc = L.orc_relax(C.byref(A), dp(f), cf.ctypes.data_as(C.POINTER(C.c_int)), rt, pts, w, 1.0, dp(l1), 1,
                     dp(u), dp(vt), dp(zt))
    assert rc == 0


@pytest.mark.parametrize("w", [1.0, 0.7])
@pytest.mark.parametrize("pts", [1, -1])
def test_cf_l1_jacobi_matches_formula(orc, w, pts):
    n = 300
    ip, jj, vv = diag_first_csr(n, 11, zero_diag_rows=(5, 77))
    keep = []
    A = orc.make_csr(ip, jj, vv, (n, n), keep)
    rng = np.random.default_rng(3)
    f, u0 = rng.standard_normal(n), rng.standard_normal(n)
    cf = np.where(rng.random(n) < 0.3, 1, -1).astype(np.int32)
    cf[5], cf[77] = pts, pts  # zero-diagonal rows of the class: skipped
    l1 = np.array([sum(abs(vv[k]) for k in range(ip[i], ip[i + 1]) if cf[jj[k]] == cf[i]) for i in range(n)])
    l1[l1 == 0] = 1.0
    u = u0.copy()
    relax(orc, A, f, cf, 18, pts, w, l1, u)
    ref = u0.copy()
    for i in range(n):
        if cf[i] != pts or vv[ip[i]] == 0.0:
            continue
        ref[i] = u0[i] + (w * row_res(ip, jj, vv, f, u0, i)) / l1[i]
    assert np.array_equal(u, ref)
    assert u[5] == u0[5] and u[77] == u0[77]
    # the other class is untouched
    other = cf != pts
    assert np.array_equal(u[other], u0[other])


def test_relax7_ignores_relax_points(orc):
    n = 200
    ip, jj, vv = diag_first_csr(n, 5)
    keep = []
    A = orc.make_csr(ip, jj, vv, (n, n), keep)
    rng = np.random.default_rng(9)
    f, u0 = rng.standard_normal(n), rng.standard_normal(n)
    cf = np.where(rng.random(n) < 0.4, 1, -1).astype(np.int32)
    d = vv[ip[:-1]].copy()
    outs = []
    for pts in (0, 1, -1):
        u = u0.copy()
        relax(orc, A, f, cf, 7, pts, 1.0, d, u)
        outs.append(u)
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[0], outs[2])
    ref = np.array([u0[i] + row_res(ip, jj, vv, f, u0, i) / d[i] for i in range(n)])
    assert np.array_equal(outs[0], ref)


def test_relax18_plain_matches_matvec_form(orc):
    n = 200
    ip, jj, vv = diag_first_csr(n, 8)
    keep = []
    A = orc.make_csr(ip, jj, vv, (n, n), keep)
    rng = np.random.default_rng(1)
    f, u0 = rng.standard_normal(n), rng.standard_normal(n)
    cf = np.ones(n, np.int32)
    l1 = np.array([sum(abs(vv[k]) for k in range(ip[i], ip[i + 1])) for i in range(n)])
    for w in (1.0, 0.6):
        u = u0.copy()
        relax(orc, A, f, cf, 18, 0, w, l1, u)
        ref = u0.copy()
        for i in range(n):
            if w == 1.0:
                v = row_res(ip, jj, vv, f, u0, i)
            else:  # csr_matvec.c: alpha=-w, beta=w -> temp=-1: t = -f + sum a u, y = -w * t
                t = -f[i]
                for k in range(ip[i], ip[i + 1]):
                    t = t + vv[k] * u0[jj[k]]
                v = -w * t
            ref[i] = u0[i] + v / l1[i]
        assert np.array_equal(u, ref), w


def test_cf_cycle_differs_from_plain(hv, orc):
    """With relax_order 1 the relax-18 cycle is C/F-ordered: it must differ
    from the relax_order 0 cycle on the same hierarchy (the l1 norms are
    C/F-restricted in both, so only the sweep order differs)."""
    A = hv.ParCSRMatrix.laplacian(14, 12, 10)
    amg = hv.BoomerAMG(**hv.ij_amg_defaults(0))
    amg.set(coarsen_type=8, relax_type=18, relax_order=1)
    amg.setup_host(A)
    O = orc.OracleAMG(amg)
    rng = np.random.default_rng(2)
    f, u0 = rng.standard_normal(A.n), rng.standard_normal(A.n)
    u_cf = u0.copy()
    O.cycle(f, u_cf)
    O.s.relax_order = 0
    u_plain = u0.copy()
    O.cycle(f, u_plain)
    assert not np.array_equal(u_cf, u_plain)
    # relax 7: relax_order 1 means two full sweeps per visit, so it differs too
    amg.set(relax_type=7)
    amg.setup_host(A)
    O7 = orc.OracleAMG(amg)
    a, b = u0.copy(), u0.copy()
    O7.cycle(f, a)
    O7.s.relax_order = 0
    O7.cycle(f, b)
    assert not np.array_equal(a, b)
