"""ctypes loader for the CPU oracle (oracle/liborc.so) -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg.  Builds the oracle's orc_amg view of a hierarchy (exported from the
product's setup through the hypreve_BoomerAMGGetLevel* introspection calls) and
runs the reference solve path (hypre_BoomerAMGCycle / Solve / PCGSolve,
restated in oracle.c) on it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liborc.so")
MAXL = 40


class orc_csr(C.Structure):
    _fields_ = [("nrows", C.c_int), ("ncols", C.c_int), ("i", C.POINTER(C.c_int)), ("j", C.POINTER(C.c_int)),
                ("a", C.POINTER(C.c_double))]


class orc_amg(C.Structure):
    _fields_ = [("num_levels", C.c_int), ("A", orc_csr * MAXL), ("P", orc_csr * MAXL),
                ("cf", C.POINTER(C.c_int) * MAXL), ("l1", C.POINTER(C.c_double) * MAXL),
                ("coarse_n", C.c_int), ("coarse_A", C.POINTER(C.c_double)),
                ("relax_type", C.c_int * 4), ("num_sweeps", C.c_int * 4),
                ("relax_weight", C.c_double), ("omega", C.c_double),
                ("relax_order", C.c_int), ("cycle_type", C.c_int), ("num_blocks", C.c_int),
                ("R", orc_csr * MAXL),
                ("cheby_ds", C.POINTER(C.c_double) * MAXL), ("cheby_coefs", (C.c_double * 5) * MAXL),
                ("cheby_order", C.c_int), ("cheby_scale", C.c_int),
                ("gs_blocks", C.POINTER(C.c_int) * MAXL), ("gs_nblocks", C.c_int * MAXL),
                ("lev_weights", C.c_int), ("lev_w", C.c_double * MAXL), ("lev_omega", C.c_double * MAXL)]


_lib = None


def build():
    subprocess.run(["make", "-s"], cwd=HERE, check=True)
    return LIB


def num_threads():
    return lib().orc_num_threads()


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        dp = C.POINTER(C.c_double)
        L.orc_matvec.argtypes = [C.c_double, C.POINTER(orc_csr), dp, C.c_double, dp, dp]
        L.orc_matvecT.argtypes = [C.c_double, C.POINTER(orc_csr), dp, C.c_double, dp]
        L.orc_relax.argtypes = [C.POINTER(orc_csr), dp, C.POINTER(C.c_int), C.c_int, C.c_int, C.c_double,
                                C.c_double, dp, C.c_int, dp, dp, dp]
        L.orc_relax.restype = C.c_int
        L.orc_cycle.argtypes = [C.POINTER(orc_amg), C.POINTER(dp), C.POINTER(dp), dp]
        L.orc_cycle.restype = C.c_int
        L.orc_amg_solve.argtypes = [C.POINTER(orc_amg), dp, dp, C.c_double, C.c_int, C.c_int, C.c_int, dp]
        L.orc_amg_solve.restype = C.c_int
        L.orc_num_threads.restype = C.c_int
        L.orc_pcg_amg.argtypes = [C.POINTER(orc_amg), dp, dp, C.c_double, C.c_int, C.c_int, dp]
        L.orc_pcg_amg.restype = C.c_int
        L.orc_dot.argtypes = [C.c_int, dp, dp]
        L.orc_dot.restype = C.c_double
        _lib = L
    return _lib


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _ip(a):
    return a.ctypes.data_as(C.POINTER(C.c_int))


def make_csr(ip, jj, vv, shape, keep):
    ip = np.ascontiguousarray(ip, dtype=np.int32)
    jj = np.ascontiguousarray(jj, dtype=np.int32)
    vv = np.ascontiguousarray(vv, dtype=np.float64)
    keep.extend([ip, jj, vv])
    return orc_csr(shape[0], shape[1], _ip(ip), _ip(jj), _dp(vv))


class OracleAMG:
    """orc_amg built from a hypreve.BoomerAMG hierarchy (after setup)."""

    def __init__(self, amg, num_blocks=None):
        self.keep = []
        s = orc_amg()
        nl = amg.num_levels()
        s.num_levels = nl
        self.n = []
        for l in range(nl):
            ip, jj, vv, shp = amg.level_matrix(l, 0)
            s.A[l] = make_csr(ip, jj, vv, shp, self.keep)
            self.n.append(shp[0])
            if l < nl - 1:
                ip, jj, vv, shp = amg.level_matrix(l, 1)
                s.P[l] = make_csr(ip, jj, vv, shp, self.keep)
                # R = P^T, rows ascending in the fine index: the restriction
                # becomes a row-parallel gather with the scatter's term order
                import scipy.sparse as sp
                R = sp.csr_matrix((vv, jj, ip), shape=shp).T.tocsr()
                R.sort_indices()
                s.R[l] = make_csr(R.indptr.astype(np.int32), R.indices.astype(np.int32),
                                  R.data.astype(np.float64), R.shape, self.keep)
            cf = amg.level_vector(l, 0)
            if cf.size:
                self.keep.append(cf)
                s.cf[l] = _ip(cf)
            l1 = amg.level_vector(l, 1)
            if l1.size:
                self.keep.append(l1)
                s.l1[l] = _dp(l1)
            gb = amg.level_vector(l, 3)
            if gb.size > 1:
                self.keep.append(gb)
                s.gs_blocks[l] = _ip(gb)
                s.gs_nblocks[l] = gb.size - 1
            if 16 in amg.relax_info()["relax_type"]:
                ds = amg.level_vector(l, 2)
                if ds.size:
                    self.keep.append(ds)
                    s.cheby_ds[l] = _dp(ds)
                co, _, prm = amg.cheby_info(l)
                for k, c in enumerate(co):
                    s.cheby_coefs[l][k] = c
                s.cheby_order, s.cheby_scale = prm[0], prm[1]
        cm = amg.coarse_matrix()
        if cm.size:
            cm = np.ascontiguousarray(cm.ravel())
            self.keep.append(cm)
            s.coarse_n = int(round(np.sqrt(cm.size)))
            s.coarse_A = _dp(cm)
        info = amg.relax_info()
        for k in range(4):
            s.relax_type[k] = info["relax_type"][k]
            s.num_sweeps[k] = info["num_sweeps"][k]
        # orc_cycle relaxes a one-level hierarchy with relax_type[0] (or 6 when
        # negative): the user relax type, par_cycle.c:296-300
        s.relax_type[0] = info["user_relax_type"]
        s.relax_weight = info["relax_weight"]
        s.omega = info["omega"]
        s.relax_order = info["relax_order"]
        s.cycle_type = info["cycle_type"]
        s.num_blocks = info["num_blocks"] if num_blocks is None else num_blocks
        s.lev_weights = 1
        for l in range(nl):
            s.lev_w[l], s.lev_omega[l] = amg.level_weights(l)
        self.s = s

    def solve(self, f, u, tol, max_iter, min_iter=0, converge_type=0):
        f = np.ascontiguousarray(f, dtype=np.float64)
        st = np.zeros(8)
        rc = lib().orc_amg_solve(C.byref(self.s), _dp(f), _dp(u), tol, min_iter, max_iter, converge_type, _dp(st))
        if rc:
            raise RuntimeError(f"oracle solve error {rc}")
        return dict(iterations=int(st[0]), rel_res=st[1], conv_factor=st[2], cycle_complexity=st[3],
                    init_res=st[4])

    def cycle(self, f, u):
        nl = self.s.num_levels
        F = (C.POINTER(C.c_double) * nl)()
        U = (C.POINTER(C.c_double) * nl)()
        bufs = []
        f = np.ascontiguousarray(f, dtype=np.float64)
        F[0] = _dp(f)
        U[0] = _dp(u)
        for l in range(1, nl):
            a, b = np.zeros(self.n[l]), np.zeros(self.n[l])
            bufs += [a, b]
            F[l] = _dp(a)
            U[l] = _dp(b)
        ops = C.c_double(0.0)
        rc = lib().orc_cycle(C.byref(self.s), F, U, C.byref(ops))
        if rc:
            raise RuntimeError(f"oracle cycle error {rc}")
        return ops.value

    def pcg(self, b, x, tol, max_iter, two_norm=1):
        b = np.ascontiguousarray(b, dtype=np.float64)
        st = np.zeros(4)
        rc = lib().orc_pcg_amg(C.byref(self.s), _dp(b), _dp(x), tol, max_iter, two_norm, _dp(st))
        if rc:
            raise RuntimeError(f"oracle pcg error {rc}")
        return int(st[0]), st[1]

    def matvec(self, level, alpha, x, beta, b):
        y = np.zeros(self.n[level])
        lib().orc_matvec(alpha, C.byref(self.s.A[level]), _dp(np.ascontiguousarray(x)), beta,
                         _dp(np.ascontiguousarray(b)), _dp(y))
        return y


def hypre_rand_stream(n, seed):
    """hypre_SeedRand(seed); n draws of hypre_Rand() (utilities/random.c)."""
    a, m = 16807, 2147483647
    s = seed if seed >= 1 else 1
    out = np.empty(n)
    for i in range(n):
        s = (a * s) % m
        out[i] = s / m
    return out
