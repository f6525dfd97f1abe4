"""Extended (interp_type 14) and extended+i (6) interpolation against a
pure-Python restatement of the reference's weight formulas, bit for bit.

Reference: src/parcsr_ls/par_lr_interp.c
* ext+i, hypre_BoomerAMGBuildExtPIInterpHost (:1041): a strong F neighbour
  k's connection a_ik is distributed over C-hat_i and i itself (the share of
  i goes to the diagonal);
* ext, hypre_BoomerAMGBuildExtInterpHost (:4686, weight loop :5194-5262):
  distributed over C-hat_i only.
Both: C-hat_i = strong C neighbours plus the strong C neighbours of strong F
neighbours, in first-touch order (:5079-5133); weak connections join the
diagonal; P_ij = w / -diagonal.  Level 0 of a 7-point Laplacian, no
truncation (P_max_elmts 0), where every off-diagonal is strong, so the
strength pattern is A's off-diagonal pattern in A's order."""
import numpy as np
import pytest

SF = -3


def ext_rows(ip, jj, vv, cf, plus_i):
    n = len(ip) - 1
    f2c = np.cumsum(cf >= 0) - 1
    out = []
    for i in range(n):
        if cf[i] >= 0:
            out.append(([int(f2c[i])], [1.0]))
            continue
        if cf[i] == SF:
            out.append(([], []))
            continue
        slot, strong_f = {}, set()
        cols, vals = [], []
        for q in range(ip[i] + 1, ip[i + 1]):  # S row i = A's off-diagonals
            i1 = jj[q]
            if cf[i1] >= 0:
                if i1 not in slot:
                    slot[i1] = len(cols)
                    cols.append(int(f2c[i1]))
                    vals.append(0.0)
            elif cf[i1] != SF:
                strong_f.add(i1)
                for r in range(ip[i1] + 1, ip[i1 + 1]):
                    k1 = jj[r]
                    if cf[k1] >= 0 and k1 not in slot:
                        slot[k1] = len(cols)
                        cols.append(int(f2c[k1]))
                        vals.append(0.0)
        diagonal = vv[ip[i]]
        for q in range(ip[i] + 1, ip[i + 1]):
            i1, a = jj[q], vv[q]
            if i1 in slot:
                vals[slot[i1]] += a
            elif i1 in strong_f:
                sgn = -1 if vv[ip[i1]] < 0 else 1
                s = 0.0
                for r in range(ip[i1] + 1, ip[i1 + 1]):
                    i2 = jj[r]
                    if (i2 in slot or (plus_i and i2 == i)) and sgn * vv[r] < 0:
                        s += vv[r]
                if s != 0:
                    d = a / s
                    for r in range(ip[i1] + 1, ip[i1 + 1]):
                        i2 = jj[r]
                        if i2 in slot and sgn * vv[r] < 0:
                            vals[slot[i2]] += d * vv[r]
                        if plus_i and i2 == i and sgn * vv[r] < 0:
                            diagonal += d * vv[r]
                else:
                    diagonal += a
            elif cf[i1] != SF:
                diagonal += a
        if diagonal:
            vals = [v / -diagonal for v in vals]
        out.append((cols, vals))
    return out


@pytest.mark.parametrize("interp_type", [14, 6])
@pytest.mark.parametrize("coarsen_type", [8, 10])
def test_ext_interp_matches_restatement(hv, interp_type, coarsen_type):
    A = hv.ParCSRMatrix.laplacian(11, 10, 9)
    amg = hv.BoomerAMG(**hv.ij_amg_defaults(0))
    amg.set(coarsen_type=coarsen_type, interp_type=interp_type, relax_type=18, P_max_elmts=0, trunc_factor=0.0)
    amg.setup_host(A)
    ip, jj, vv, _ = amg.level_matrix(0, 0)
    cf = amg.level_vector(0, 0).astype(np.int64)
    pi, pj, pv, _ = amg.level_matrix(0, 1)
    rows = ext_rows(ip, jj, vv, cf, plus_i=interp_type == 6)
    assert len(rows) == len(pi) - 1
    for i, (cols, vals) in enumerate(rows):
        got_j = pj[pi[i]:pi[i + 1]].tolist()
        got_v = pv[pi[i]:pi[i + 1]]
        assert got_j == cols, i
        assert np.array_equal(got_v, np.array(vals, dtype=np.float64)), i


def test_ext_differs_from_ext_plus_i(hv):
    A = hv.ParCSRMatrix.laplacian(11, 10, 9)
    P = {}
    for t in (6, 14):
        amg = hv.BoomerAMG(**hv.ij_amg_defaults(0))
        amg.set(coarsen_type=8, interp_type=t, relax_type=18, P_max_elmts=0, trunc_factor=0.0)
        amg.setup_host(A)
        P[t] = amg.level_matrix(0, 1)
    assert np.array_equal(P[6][0], P[14][0]) and np.array_equal(P[6][1], P[14][1])
    assert not np.array_equal(P[6][2], P[14][2])


def test_ext_interp_solves(hv):
    """The ext hierarchy converges as a preconditioner (setup + host checks
    only; the GPU band against gpu_boomer.saved out.15 is in test_gpu_scale)."""
    A = hv.ParCSRMatrix.laplacian(20, 20, 20)
    amg = hv.BoomerAMG(**hv.ij_amg_defaults(0))
    amg.set(coarsen_type=8, interp_type=14, relax_type=18, P_max_elmts=4)
    amg.setup_host(A)
    g, o, _ = amg.complexities()
    assert 1.0 < g < 2.0 and 1.0 < o < 4.0


def modextpe_rows(ip, jj, vv, cf):
    """par_mod_lr_interp.c:1040 (ext+e, matrix-matrix form), one process:
    As_FF / As_FC as gen_fffc.c:19, W = As_FF As_FC as par_csr_matop.c:277."""
    n = len(ip) - 1
    fr = [i for i in range(n) if cf[i] <= 0]
    f2f = {i: r for r, i in enumerate(fr)}
    f2c = {}
    for i in range(n):
        if cf[i] > 0:
            f2c[i] = len(f2c)
    nF, nC = len(fr), len(f2c)
    FF, FC = [], []
    for i in fr:
        ff = [[f2f[i], vv[ip[i]]]]
        fc = []
        for q in range(ip[i] + 1, ip[i + 1]):  # S row i = A's off-diagonals here
            j = jj[q]
            (fc if cf[j] > 0 else ff).append([f2c[j] if cf[j] > 0 else f2f[j], vv[q]])
        FF.append(ff)
        FC.append(fc)
    lam, beta, tmp = [0.0] * nF, [0.0] * nF, [0.0] * nF
    for r in range(nF):
        for _, a in FF[r][1:]:
            lam[r] += a
        number = float(len(FF[r]) - 1)
        if number:
            lam[r] /= number
        for _, a in FC[r]:
            beta[r] += a
        if lam[r] + beta[r]:
            tmp[r] = lam[r] / (beta[r] + lam[r])
    dw, tau = [0.0] * nF, [0.0] * nF
    for r, i in enumerate(fr):
        for q in range(ip[i], ip[i + 1]):
            dw[r] += vv[q]
        for _, a in FF[r][1:]:
            dw[r] -= a
        dw[r] -= beta[r]
        for c, a in FF[r][1:]:
            tau[r] += a * tmp[c]
    for r in range(nF):
        value = dw[r] + tau[r]
        if value:
            value = -1.0 / value
        theta = beta[r] + lam[r]
        FF[r][0][1] = value * theta
        if theta:
            theta = 1.0 / theta
        for e in FF[r][1:]:
            e[1] *= value
        for e in FC[r]:
            e[1] *= theta
    rows, W = [], []
    for r in range(nF):
        cols, vals, slot = [], [], {}
        if nF == nC:
            slot[r] = 0
            cols.append(r)
            vals.append(0.0)
        for k, a in FF[r]:
            for c, b in FC[k]:
                if c not in slot:
                    slot[c] = len(cols)
                    cols.append(c)
                    vals.append(a * b)
                else:
                    vals[slot[c]] += a * b
        W.append((cols, vals))
    for i in range(n):
        rows.append(([f2c[i]], [1.0]) if cf[i] > 0 else W[f2f[i]])
    return rows


@pytest.mark.parametrize("coarsen_type", [8, 10])
@pytest.mark.parametrize("dims", [(11, 10, 9), (7, 6, 5)])
def test_modextpe_interp_matches_restatement(hv, coarsen_type, dims):
    A = hv.ParCSRMatrix.laplacian(*dims)
    amg = hv.BoomerAMG(**hv.ij_amg_defaults(0))
    amg.set(coarsen_type=coarsen_type, interp_type=18, relax_type=18, P_max_elmts=0, trunc_factor=0.0)
    amg.setup_host(A)
    ip, jj, vv, _ = amg.level_matrix(0, 0)
    cf = amg.level_vector(0, 0).astype(np.int64)
    pi, pj, pv, _ = amg.level_matrix(0, 1)
    rows = modextpe_rows(ip, jj, vv, cf)
    assert len(rows) == len(pi) - 1
    for i, (cols, vals) in enumerate(rows):
        assert pj[pi[i]:pi[i + 1]].tolist() == cols, i
        assert np.array_equal(pv[pi[i]:pi[i + 1]], np.array(vals, dtype=np.float64)), i


def _fffc(ip, jj, vv, cf, partial):
    """gen_fffc.c:19 (partial False) / :506 GenerateFFFC3 (partial True) on a
    matrix whose strength pattern is its off-diagonal pattern."""
    n = len(ip) - 1
    f2f, f2c = {}, {}
    for i in range(n):
        if cf[i] > 0:
            f2c[i] = len(f2c)
        else:
            f2f[i] = len(f2f)
    frow = [i for i in range(n) if cf[i] < 0]
    ffrow = [i for i in range(n) if (cf[i] == -2 if partial else cf[i] < 0)]
    FC = [[[f2c[jj[q]], vv[q]] for q in range(ip[i] + 1, ip[i + 1]) if cf[jj[q]] > 0] for i in frow]
    FF = [[[f2f[i], vv[ip[i]]]] + [[f2f[jj[q]], vv[q]] for q in range(ip[i] + 1, ip[i + 1]) if cf[jj[q]] <= 0]
          for i in ffrow]
    return FF, FC, frow, ffrow, len(f2c)


def _matmul(X, Y, ncols):
    out = []
    for r, row in enumerate(X):
        cols, vals, slot = [], [], {}
        if len(X) == ncols:
            slot[r] = 0
            cols.append(r)
            vals.append(0.0)
        for k, a in row:
            for c, b in Y[k]:
                if c not in slot:
                    slot[c] = len(cols)
                    cols.append(c)
                    vals.append(a * b)
                else:
                    vals[slot[c]] += a * b
        out.append([[c, v] for c, v in zip(cols, vals)])
    return out


def modext_rows(ip, jj, vv, cf):
    """par_mod_lr_interp.c:16 hypre_BoomerAMGBuildModExtInterpHost."""
    FF, FC, frow, _, nC = _fffc(ip, jj, vv, cf, False)
    for r, i in enumerate(frow):
        dq = 0.0
        for _, a in FC[r]:
            dq += a
        dw = 0.0
        for q in range(ip[i], ip[i + 1]):
            dw += vv[q]
        for _, a in FF[r][1:]:
            dw -= a
        dw -= dq
        beta = 1.0 / dw if dw else 1.0
        FF[r][0][1] = beta * dq
        gamma = -1.0 / dq if dq else 1.0
        for e in FF[r][1:]:
            e[1] *= beta
        for e in FC[r]:
            e[1] *= gamma
    W = _matmul(FF, FC, nC)
    it = iter(W)
    return [[[c, 1.0]] if cf[i] > 0 else next(it) for i, c in
            ((i, sum(1 for k in range(i) if cf[k] > 0)) for i in range(len(ip) - 1))]


def modpartialext_rows(ip, jj, vv, cf, pe=False):
    """par_2s_interp.c:15 hypre_BoomerAMGBuildModPartialExtInterpHost; pe:
    :564 hypre_BoomerAMGBuildModPartialExtPEInterpHost (D_lambda as
    gen_fffc.c:1056 GenerateFFFCD3)."""
    FF, FC, frow, ffrow, nC = _fffc(ip, jj, vv, cf, True)
    fidx = {i: r for r, i in enumerate(frow)}
    dq, lam, dinv = [], [], []
    for r, row in enumerate(FC):
        s = 0.0
        for _, a in row:
            s += a
        dq.append(s)
        i = frow[r]
        lm, cnt = 0.0, 0
        for q in range(ip[i] + 1, ip[i + 1]):
            if cf[jj[q]] <= 0:
                cnt += 1
                lm += vv[q]
        if cnt:
            lm = lm / cnt
        lam.append(lm)
        dinv.append(1.0 / (s + lm) if s + lm else 0.0)
    for r, i in enumerate(ffrow):
        fi = fidx[i]
        dw = 0.0
        if pe:
            tau = 0.0
            for c, a in FF[r][1:]:
                tau += a * lam[c] * dinv[c]
            for q in range(ip[i], ip[i + 1]):
                dw += vv[q]
            for c, a in FF[r][1:]:
                if dinv[c]:
                    dw -= a
            dw += tau - dq[fi]
        else:
            for q in range(ip[i], ip[i + 1]):
                dw += vv[q]
            for c, a in FF[r][1:]:
                if dq[c]:
                    dw -= a
            dw -= dq[fi]
        if dw:
            b = -1.0 / dw if pe else 1.0 / dw
            FF[r][0][1] = b * (dq[fi] + lam[fi]) if pe else b * dq[fi]
            for e in FF[r][1:]:
                e[1] *= b
    for r in range(len(FC)):
        g = dinv[r] if pe else (-1.0 / dq[r] if dq[r] else 0.0)
        for e in FC[r]:
            e[1] *= g
    W = _matmul(FF, FC, nC)
    it = iter(W)
    rows, c = [], 0
    for i in range(len(ip) - 1):
        if cf[i] > 0:
            rows.append([[c, 1.0]])
            c += 1
        elif cf[i] == -2:
            rows.append(next(it))
    return rows


@pytest.mark.parametrize("agg_interp", [5, 7])
@pytest.mark.parametrize("coarsen_type", [8, 10])
def test_two_stage_modext_agg_interp_matches_restatement(hv, coarsen_type, agg_interp):
    """agg_interp_type 5 / 7 (par_amg_setup.c:1575-1689): P = P1 P2 with P1
    the extended (ext+e) MM interpolation to the first pass's C points and P2
    the partial one from them to the second pass's; no truncation."""
    A = hv.ParCSRMatrix.laplacian(14, 13, 12)
    amg = hv.BoomerAMG(**hv.ij_amg_defaults(0))
    amg.set(coarsen_type=coarsen_type, relax_type=18, agg_num_levels=1, agg_interp_type=agg_interp,
            agg_P_max_elmts=0, agg_P12_max_elmts=0, agg_trunc_factor=0.0, agg_P12_trunc_factor=0.0)
    amg.setup_host(A)
    ip, jj, vv, _ = amg.level_matrix(0, 0)
    cf = amg.level_vector(0, 0).astype(np.int64)
    assert (cf == -2).any() and (cf == 1).any()
    cf1 = np.where(cf == -2, 1, cf)
    if agg_interp == 5:
        P1 = modext_rows(ip, jj, vv, cf1)
    else:
        P1 = [[[c, v] for c, v in zip(*row)] for row in modextpe_rows(ip, jj, vv, cf1)]
    P2 = modpartialext_rows(ip, jj, vv, cf, pe=agg_interp == 7)
    P = _matmul(P1, P2, int((cf == 1).sum()))
    pi, pj, pv, _ = amg.level_matrix(0, 1)
    assert len(P) == len(pi) - 1
    for i, row in enumerate(P):
        assert pj[pi[i]:pi[i + 1]].tolist() == [c for c, _ in row], i
        assert np.array_equal(pv[pi[i]:pi[i + 1]], np.array([v for _, v in row], dtype=np.float64)), i


def modextpi_rows(ip, jj, vv, cf):
    """par_mod_lr_interp.c:474 hypre_BoomerAMGBuildModExtPIInterpHost."""
    FF, FC, frow, _, nC = _fffc(ip, jj, vv, cf, False)
    orig = [[e[1] for e in row] for row in FF]
    dq = []
    for row in FC:
        s = 0.0
        for _, a in row:
            s += a
        dq.append(s)
    dw = []
    for r, i in enumerate(frow):
        w = 0.0
        for q in range(ip[i], ip[i + 1]):
            w += vv[q]
        for _, a in FF[r][1:]:
            w -= a
        w -= dq[r]
        dw.append(w)
    for r in range(len(FF)):
        th = 0.0
        for e in FF[r][1:]:
            c = e[0]
            value = dq[c]
            for k in range(1, len(FF[c])):
                if FF[c][k][0] == r:
                    value1 = orig[c][k]
                    value += value1
                    th += e[1] * value1 / value
                    break
            e[1] /= value
        FF[r][0][1] = 1.0
        theta = th + dw[r]
        if theta:
            theta = -1.0 / theta
            for e in FF[r]:
                e[1] *= theta
    W = _matmul(FF, FC, nC)
    it = iter(W)
    rows, c = [], 0
    for i in range(len(ip) - 1):
        if cf[i] > 0:
            rows.append([[c, 1.0]])
            c += 1
        else:
            rows.append(next(it))
    return rows


@pytest.mark.parametrize("interp_type", [16, 17])
@pytest.mark.parametrize("coarsen_type", [8, 10])
def test_modext_modextpi_interp_matches_restatement(hv, interp_type, coarsen_type):
    """interp_type 16 (par_mod_lr_interp.c:16) and 17 (:474), no truncation."""
    A = hv.ParCSRMatrix.laplacian(11, 10, 9)
    amg = hv.BoomerAMG(**hv.ij_amg_defaults(0))
    amg.set(coarsen_type=coarsen_type, interp_type=interp_type, relax_type=18, P_max_elmts=0, trunc_factor=0.0)
    amg.setup_host(A)
    ip, jj, vv, _ = amg.level_matrix(0, 0)
    cf = amg.level_vector(0, 0).astype(np.int64)
    rows = (modext_rows if interp_type == 16 else modextpi_rows)(ip, jj, vv, cf)
    pi, pj, pv, _ = amg.level_matrix(0, 1)
    assert len(rows) == len(pi) - 1
    for i, row in enumerate(rows):
        assert pj[pi[i]:pi[i + 1]].tolist() == [c for c, _ in row], i
        assert np.array_equal(pv[pi[i]:pi[i + 1]], np.array([v for _, v in row], dtype=np.float64)), i
