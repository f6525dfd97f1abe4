"""Inputs of the reference's np > 1 `ij` runs, rebuilt for one process.

Test infrastructure: the matrix and right-hand side that `mpirun -np N ./ij
-P p q r [-27pt] [-rhsrand]` builds (test/ij.c BuildParLaplacian[27pt],
parcsr_ls/par_laplace.c:15 / par_laplace_27pt.c, hypre_GeneratePartitioning),
stacked rank by rank.  Rows are in rank order and each row keeps its
generation order; hypreve_BoomerAMGSetRankEmulation puts every row into ParCSR
order (own columns first) and emulates the per-rank coarsening.
"""
import math

import numpy as np
import scipy.sparse as sp


def partition(n, p):
    """hypre_GeneratePartitioning: p pieces of n, the first n % p one longer."""
    size, rest = n // p, n % p
    return [i * size + min(i, rest) for i in range(p + 1)]


def laplacian_ranks(nx, ny, nz, P, Q, R, c=(1.0, 1.0, 1.0), pt27=False):
    """(scipy CSR, level-0 rank starts) of GenerateLaplacian / GenerateLaplacian27pt
    on a P x Q x R process grid; rank = p + P*q + P*Q*r."""
    xp, yp, zp = partition(nx, P), partition(ny, Q), partition(nz, R)
    own_x = np.searchsorted(xp, np.arange(nx), side="right") - 1
    own_y = np.searchsorted(yp, np.arange(ny), side="right") - 1
    own_z = np.searchsorted(zp, np.arange(nz), side="right") - 1
    offs = {}
    o = 0
    for r in range(R):
        for q in range(Q):
            for p in range(P):
                offs[p + P * q + P * Q * r] = o
                o += (xp[p + 1] - xp[p]) * (yp[q + 1] - yp[q]) * (zp[r + 1] - zp[r])

    def gidx(ix, iy, iz):
        p, q, r = own_x[ix], own_y[iy], own_z[iz]
        nxl, nyl = xp[p + 1] - xp[p], yp[q + 1] - yp[q]
        return offs[p + P * q + P * Q * r] + (ix - xp[p]) + nxl * ((iy - yp[q]) + nyl * (iz - zp[r]))

    cx, cy, cz = c
    v0 = (2 * cx if nx > 1 else 0.0) + (2 * cy if ny > 1 else 0.0) + (2 * cz if nz > 1 else 0.0)
    ip, jj, vv, starts = [0], [], [], [0]
    for rk in range(P * Q * R):
        p, q, r = rk % P, (rk // P) % Q, rk // (P * Q)
        for iz in range(zp[r], zp[r + 1]):
            for iy in range(yp[q], yp[q + 1]):
                for ix in range(xp[p], xp[p + 1]):
                    row = gidx(ix, iy, iz)
                    if pt27:
                        ent = [(row, 26.0)]
                        for dz in (-1, 0, 1):
                            for dy in (-1, 0, 1):
                                for dx in (-1, 0, 1):
                                    jx, jy, jz = ix + dx, iy + dy, iz + dz
                                    if (dx or dy or dz) and 0 <= jx < nx and 0 <= jy < ny and 0 <= jz < nz:
                                        ent.append((gidx(jx, jy, jz), -1.0))
                    else:
                        ent = [(row, v0)]
                        for jx, jy, jz, v in ((ix, iy, iz - 1, -cz), (ix, iy - 1, iz, -cy), (ix - 1, iy, iz, -cx),
                                              (ix + 1, iy, iz, -cx), (ix, iy + 1, iz, -cy), (ix, iy, iz + 1, -cz)):
                            if 0 <= jx < nx and 0 <= jy < ny and 0 <= jz < nz:
                                ent.append((gidx(jx, jy, jz), v))
                    for col, v in ent:
                        jj.append(col)
                        vv.append(v)
                    ip.append(len(jj))
        starts.append(len(ip) - 1)
    n = nx * ny * nz
    A = sp.csr_matrix((np.array(vv), np.array(jj, dtype=np.int32), np.array(ip, dtype=np.int32)), shape=(n, n))
    return A, starts


def sys_laplacian_ranks(nx, ny, nz, P, Q, R, nf=3, mtrx=None):
    """(scipy CSR, level-0 rank starts) of ij -sysL nf (BuildParSysLaplacian,
    sys_opt 0; par_laplace.c:394 GenerateSysLaplacian) on a P x Q x R process
    grid: nf interleaved unknowns a grid point, row (point, f) holding the
    blocks own, z-1, y-1, x-1, x+1, y+1, z+1 of nf entries each (value[k] *
    mtrx[f][j], zeros stored), the own block's entries 0 and f swapped so the
    diagonal comes first (par_laplace.c:846-860)."""
    if mtrx is None:
        mtrx = {2: [2.0, 1.0, 1.0, 2.0], 3: [2.0, 1.0, 0.0, 1.0, 2.0, 1.0, 0.0, 1.0, 2.0]}[nf]
    xp, yp, zp = partition(nx, P), partition(ny, Q), partition(nz, R)
    own_x = np.searchsorted(xp, np.arange(nx), side="right") - 1
    own_y = np.searchsorted(yp, np.arange(ny), side="right") - 1
    own_z = np.searchsorted(zp, np.arange(nz), side="right") - 1
    offs = {}
    o = 0
    for r in range(R):
        for q in range(Q):
            for p in range(P):
                offs[p + P * q + P * Q * r] = o
                o += (xp[p + 1] - xp[p]) * (yp[q + 1] - yp[q]) * (zp[r + 1] - zp[r])

    def gidx(ix, iy, iz):
        p, q, r = own_x[ix], own_y[iy], own_z[iz]
        nxl, nyl = xp[p + 1] - xp[p], yp[q + 1] - yp[q]
        return offs[p + P * q + P * Q * r] + (ix - xp[p]) + nxl * ((iy - yp[q]) + nyl * (iz - zp[r]))

    value = [0.0, -1.0, -1.0, -1.0]
    for dim in (nx, ny, nz):
        if dim > 1:
            value[0] += 2.0
    ip, jj, vv, starts = [0], [], [], [0]
    for rk in range(P * Q * R):
        p, q, r = rk % P, (rk // P) % Q, rk // (P * Q)
        for iz in range(zp[r], zp[r + 1]):
            for iy in range(yp[q], yp[q + 1]):
                for ix in range(xp[p], xp[p + 1]):
                    blocks = [(gidx(ix, iy, iz), 0)]
                    for jx, jy, jz, k in ((ix, iy, iz - 1, 3), (ix, iy - 1, iz, 2), (ix - 1, iy, iz, 1),
                                          (ix + 1, iy, iz, 1), (ix, iy + 1, iz, 2), (ix, iy, iz + 1, 3)):
                        if 0 <= jx < nx and 0 <= jy < ny and 0 <= jz < nz:
                            blocks.append((gidx(jx, jy, jz), k))
                    for f in range(nf):
                        ent = []
                        for g, k in blocks:
                            for j in range(nf):
                                ent.append((nf * g + j, value[k] * mtrx[f * nf + j]))
                        ent[0], ent[f] = ent[f], ent[0]
                        for col, v in ent:
                            jj.append(col)
                            vv.append(v)
                        ip.append(len(jj))
        starts.append(len(ip) - 1)
    n = nf * nx * ny * nz
    A = sp.csr_matrix((np.array(vv), np.array(jj, dtype=np.int32), np.array(ip, dtype=np.int32)), shape=(n, n))
    return A, starts


def rotate_ranks(nx, ny, P, Q, alpha, eps):
    """(scipy CSR, level-0 rank starts) of ij -rotate (BuildParRotate7pt,
    parcsr_ls/par_rotate_7pt.c GenerateRotate7pt) on a P x Q process grid,
    rank = p + P*q: the rotated anisotropic 2-D operator, each row centre,
    (-1,-1), (0,-1), (-1,0), (+1,0), (0,+1), (+1,+1)."""
    x = 4.0 * math.atan(1.0) * alpha / 180.0
    s, c = math.sin(x), math.cos(x)
    ac = -(c * c + eps * s * s)
    bc = 2.0 * (1.0 - eps) * s * c
    cc = -(s * s + eps * c * c)
    v0, v1, v2, v3 = -2 * (2 * ac + bc + 2 * cc), 2 * ac + bc, bc + 2 * cc, -bc
    xp, yp = partition(nx, P), partition(ny, Q)
    own_x = np.searchsorted(xp, np.arange(nx), side="right") - 1
    own_y = np.searchsorted(yp, np.arange(ny), side="right") - 1
    offs, o = {}, 0
    for q in range(Q):
        for p in range(P):
            offs[p + P * q] = o
            o += (xp[p + 1] - xp[p]) * (yp[q + 1] - yp[q])

    def gidx(ix, iy):
        p, q = own_x[ix], own_y[iy]
        return offs[p + P * q] + (ix - xp[p]) + (xp[p + 1] - xp[p]) * (iy - yp[q])

    ip, jj, vv, starts = [0], [], [], [0]
    for rk in range(P * Q):
        p, q = rk % P, rk // P
        for iy in range(yp[q], yp[q + 1]):
            for ix in range(xp[p], xp[p + 1]):
                ent = [(gidx(ix, iy), v0)]
                for jx, jy, v in ((ix - 1, iy - 1, v3), (ix, iy - 1, v2), (ix - 1, iy, v1), (ix + 1, iy, v1),
                                  (ix, iy + 1, v2), (ix + 1, iy + 1, v3)):
                    if 0 <= jx < nx and 0 <= jy < ny:
                        ent.append((gidx(jx, jy), v))
                for col, v in ent:
                    jj.append(col)
                    vv.append(v)
                ip.append(len(jj))
        starts.append(len(ip) - 1)
    n = nx * ny
    A = sp.csr_matrix((np.array(vv), np.array(jj, dtype=np.int32), np.array(ip, dtype=np.int32)), shape=(n, n))
    return A, starts


def _vdc_coef(xx, yy, zz):
    """afun = bfun = cfun of par_vardifconv.c:397-483: 0.01 in the eight corner
    cubes, 1000 in the inner cube, 1 elsewhere."""
    lo = lambda v: v < 0.1
    hi = lambda v: v > 0.9
    if ((lo(xx) and lo(yy) and lo(zz)) or (lo(xx) and lo(yy) and hi(zz)) or (lo(xx) and hi(yy) and lo(zz))
            or (hi(xx) and lo(yy) and lo(zz)) or (hi(xx) and hi(yy) and lo(zz)) or (hi(xx) and lo(yy) and hi(zz))
            or (lo(xx) and hi(yy) and hi(zz)) or (hi(xx) and hi(yy) and hi(zz))):
        return 0.01
    if 0.1 <= xx <= 0.9 and 0.1 <= yy <= 0.9 and 0.1 <= zz <= 0.9:
        return 1000.0
    return 1.0


def vardifconv_ranks(nx, ny, nz, P, Q, R, eps):
    """(scipy CSR, level-0 rank starts, rhs) of ij -vardifconv (type 0,
    parcsr_ls/par_vardifconv.c:15 GenerateVarDifConv) on a P x Q x R process
    grid: the variable-coefficient diffusion with d = e = f = g = 0, r = 1 and
    zero boundary values, each row centre, z-1, y-1, x-1, x+1, y+1, z+1."""
    xp, yp, zp = partition(nx, P), partition(ny, Q), partition(nz, R)
    own_x = np.searchsorted(xp, np.arange(nx), side="right") - 1
    own_y = np.searchsorted(yp, np.arange(ny), side="right") - 1
    own_z = np.searchsorted(zp, np.arange(nz), side="right") - 1
    offs, o = {}, 0
    for r in range(R):
        for q in range(Q):
            for p in range(P):
                offs[p + P * q + P * Q * r] = o
                o += (xp[p + 1] - xp[p]) * (yp[q + 1] - yp[q]) * (zp[r + 1] - zp[r])

    def gidx(ix, iy, iz):
        p, q, r = own_x[ix], own_y[iy], own_z[iz]
        nxl, nyl = xp[p + 1] - xp[p], yp[q + 1] - yp[q]
        return offs[p + P * q + P * Q * r] + (ix - xp[p]) + nxl * ((iy - yp[q]) + nyl * (iz - zp[r]))

    hhx, hhy, hhz = 1.0 / (nx + 1), 1.0 / (ny + 1), 1.0 / (nz + 1)
    ip, jj, vv, rhs, starts = [0], [], [], [], [0]
    for rk in range(P * Q * R):
        p, q, r = rk % P, (rk // P) % Q, rk // (P * Q)
        for iz in range(zp[r], zp[r + 1]):
            zz = (iz + 1) * hhz
            for iy in range(yp[q], yp[q + 1]):
                yy = (iy + 1) * hhy
                for ix in range(xp[p], xp[p + 1]):
                    xx = (ix + 1) * hhx
                    afp = eps * _vdc_coef(xx + 0.5 * hhx, yy, zz) / hhx / hhx
                    afm = eps * _vdc_coef(xx - 0.5 * hhx, yy, zz) / hhx / hhx
                    bfp = eps * _vdc_coef(xx, yy + 0.5 * hhy, zz) / hhy / hhy
                    bfm = eps * _vdc_coef(xx, yy - 0.5 * hhy, zz) / hhy / hhy
                    cfp = eps * _vdc_coef(xx, yy, zz + 0.5 * hhz) / hhz / hhz
                    cfm = eps * _vdc_coef(xx, yy, zz - 0.5 * hhz) / hhz / hhz
                    df = ef = ff = gf = 0.0
                    ent = [(gidx(ix, iy, iz), afp + afm + bfp + bfm + cfp + cfm + gf - df - ef - ff)]
                    # rfun = 1; the boundary terms add coefficient * bndfun = 0
                    b = 1.0
                    for cond, coef in ((ix == 0, afm), (iy == 0, bfm), (iz == 0, cfm), (ix + 1 == nx, afp - df),
                                       (iy + 1 == ny, bfp - ef), (iz + 1 == nz, cfp - ff)):
                        if cond:
                            b += coef * 0.0
                    rhs.append(b)
                    for jx, jy, jz, v in ((ix, iy, iz - 1, -cfm), (ix, iy - 1, iz, -bfm), (ix - 1, iy, iz, -afm),
                                          (ix + 1, iy, iz, -afp + df), (ix, iy + 1, iz, -bfp + ef),
                                          (ix, iy, iz + 1, -cfp + ff)):
                        if 0 <= jx < nx and 0 <= jy < ny and 0 <= jz < nz:
                            ent.append((gidx(jx, jy, jz), v))
                    for col, v in ent:
                        jj.append(col)
                        vv.append(v)
                    ip.append(len(jj))
        starts.append(len(ip) - 1)
    n = nx * ny * nz
    A = sp.csr_matrix((np.array(vv), np.array(jj, dtype=np.int32), np.array(ip, dtype=np.int32)), shape=(n, n))
    return A, starts, np.array(rhs)


def rand_guess(starts):
    """ij's random initial guess (build_src_type 5, ij.c:3046): every rank
    hypre_SeedRand(myid), then hypre_Rand() per entry."""
    return np.concatenate([rand_stream(starts[k + 1] - starts[k], k) for k in range(len(starts) - 1)])


def rand_stream(n, seed):
    """n draws of hypre_Rand() after hypre_SeedRand(seed) (utilities/random.c)."""
    a, m = 16807, 2147483647
    s = seed if seed >= 1 else 1
    out = np.empty(n)
    for i in range(n):
        s = (a * s) % m
        out[i] = s / m
    return out


def rhsrand(starts):
    """ij -rhsrand (ij.c:2750): HYPRE_ParVectorSetRandomValues(b, 22775), every
    rank seeding 22775 * (rank + 1) (par_vector.c:337), then b /= ||b||."""
    b = np.concatenate([2.0 * rand_stream(starts[k + 1] - starts[k], 22775 * (k + 1)) - 1.0
                        for k in range(len(starts) - 1)])
    return b * (1.0 / np.sqrt(np.dot(b, b)))
