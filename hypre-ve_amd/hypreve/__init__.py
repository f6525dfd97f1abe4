"""Python binding of libhypreve.so (the C ABI in include/hypreve.h).

This mirrors the reference's C interface one-to-one (HYPRE_IJ*, HYPRE_ParCSR*,
HYPRE_BoomerAMG*, HYPRE_ParCSRPCG*, GenerateLaplacian) so tests and the bench
drive the product exactly as a hypre user's C code would.  It adds no compute
of its own: every solve-path operation runs in the HIP kernels of the library.
The library refuses to run a solve without a GPU (HYPRE_Init fails), there is
no CPU fallback.

Reference: src/parcsr_ls/HYPRE_parcsr_ls.h, src/IJ_mv/HYPRE_IJ_mv.h,
src/krylov/HYPRE_krylov.h (SX-Aurora/hypre-ve).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
LIB_PATH = os.path.join(PKG_ROOT, "lib", "libhypreve.so")

HYPRE_PARCSR = 5555
HYPRE_MEMORY_HOST = 0
HYPRE_MEMORY_DEVICE = 1
HYPRE_ERROR_GENERIC = 1
HYPRE_ERROR_ARG = 4
HYPRE_ERROR_CONV = 256

_lib = None


def build(force: bool = False) -> str:
    """Compile libhypreve.so in-tree (hipcc --offload-arch=gfx950)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-j8"], cwd=PKG_ROOT, check=True)
    return LIB_PATH


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: run `make -C hypre-ve_amd` (no fallback path exists)")
        # HVE_LIB_PATH: another build of the same sources (A/B experiments on
        # compile-time variants); the default is the in-tree library
        _lib = C.CDLL(os.environ.get("HVE_LIB_PATH", LIB_PATH), mode=C.RTLD_GLOBAL)
        _declare(_lib)
    return _lib


_p = C.c_void_p
_i = C.c_int
_d = C.c_double
_pi = C.POINTER(C.c_int)
_pd = C.POINTER(C.c_double)
_pi64 = C.POINTER(C.c_int64)

SOLVER_FCN = C.CFUNCTYPE(_i, _p, _p, _p, _p)

# (name, restype, argtypes) for every symbol include/hypreve.h declares
SIGNATURES = [
    ("HYPRE_Init", _i, []),
    ("HYPRE_Finalize", _i, []),
    ("HYPRE_SetMemoryLocation", _i, [_i]),
    ("HYPRE_GetError", _i, []),
    ("HYPRE_ClearAllErrors", _i, []),
    ("HYPRE_CheckError", _i, [_i, _i]),
    ("HYPRE_IJMatrixCreate", _i, [_p, _i, _i, _i, _i, C.POINTER(_p)]),
    ("HYPRE_IJMatrixDestroy", _i, [_p]),
    ("HYPRE_IJMatrixInitialize", _i, [_p]),
    ("HYPRE_IJMatrixSetObjectType", _i, [_p, _i]),
    ("HYPRE_IJMatrixSetValues", _i, [_p, _i, _pi, _pi, _pi, _pd]),
    ("HYPRE_IJMatrixAddToValues", _i, [_p, _i, _pi, _pi, _pi, _pd]),
    ("HYPRE_IJMatrixAssemble", _i, [_p]),
    ("HYPRE_IJMatrixGetObject", _i, [_p, C.POINTER(_p)]),
    ("HYPRE_IJVectorCreate", _i, [_p, _i, _i, C.POINTER(_p)]),
    ("HYPRE_IJVectorDestroy", _i, [_p]),
    ("HYPRE_IJVectorInitialize", _i, [_p]),
    ("HYPRE_IJVectorSetObjectType", _i, [_p, _i]),
    ("HYPRE_IJVectorSetValues", _i, [_p, _i, _pi, _pd]),
    ("HYPRE_IJVectorGetValues", _i, [_p, _i, _pi, _pd]),
    ("HYPRE_IJVectorAssemble", _i, [_p]),
    ("HYPRE_IJVectorGetObject", _i, [_p, C.POINTER(_p)]),
    ("HYPRE_ParCSRMatrixDestroy", _i, [_p]),
    ("HYPRE_ParCSRMatrixGetLocalRange", _i, [_p, _pi, _pi, _pi, _pi]),
    ("HYPRE_ParCSRMatrixMatvec", _i, [_d, _p, _p, _d, _p]),
    ("HYPRE_ParCSRMatrixMatvecOutOfPlace", _i, [_d, _p, _p, _d, _p, _p]),
    ("HYPRE_ParCSRMatrixMatvecT", _i, [_d, _p, _p, _d, _p]),
    ("HYPRE_ParVectorCreate", _i, [_p, _i, _pi, C.POINTER(_p)]),
    ("HYPRE_ParVectorInitialize", _i, [_p]),
    ("HYPRE_ParVectorDestroy", _i, [_p]),
    ("HYPRE_ParVectorSetConstantValues", _i, [_p, _d]),
    ("HYPRE_ParVectorCopy", _i, [_p, _p]),
    ("HYPRE_ParVectorScale", _i, [_d, _p]),
    ("HYPRE_ParVectorAxpy", _i, [_d, _p, _p]),
    ("HYPRE_ParVectorInnerProd", _i, [_p, _p, _pd]),
    ("GenerateLaplacian", _p, [_p, _i, _i, _i, _i, _i, _i, _i, _i, _i, _pd]),
    ("GenerateLaplacian27pt", _p, [_p, _i, _i, _i, _i, _i, _i, _i, _i, _i, _pd]),
    ("HYPRE_BoomerAMGCreate", _i, [C.POINTER(_p)]),
    ("HYPRE_BoomerAMGDestroy", _i, [_p]),
    ("HYPRE_BoomerAMGSetup", _i, [_p, _p, _p, _p]),
    ("HYPRE_BoomerAMGSolve", _i, [_p, _p, _p, _p]),
    ("HYPRE_BoomerAMGGetNumIterations", _i, [_p, _pi]),
    ("HYPRE_BoomerAMGGetFinalRelativeResidualNorm", _i, [_p, _pd]),
    ("HYPRE_BoomerAMGSetConvergeType", _i, [_p, _i]),
    ("HYPRE_BoomerAMGSetTol", _i, [_p, _d]),
    ("HYPRE_BoomerAMGSetMaxIter", _i, [_p, _i]),
    ("HYPRE_BoomerAMGSetMinIter", _i, [_p, _i]),
    ("HYPRE_BoomerAMGSetMaxCoarseSize", _i, [_p, _i]),
    ("HYPRE_BoomerAMGSetMinCoarseSize", _i, [_p, _i]),
    ("HYPRE_BoomerAMGSetMaxLevels", _i, [_p, _i]),
    ("HYPRE_BoomerAMGSetStrongThreshold", _i, [_p, _d]),
    ("HYPRE_BoomerAMGSetMaxRowSum", _i, [_p, _d]),
    ("HYPRE_BoomerAMGSetCoarsenType", _i, [_p, _i]),
    ("HYPRE_BoomerAMGSetMeasureType", _i, [_p, _i]),
    ("HYPRE_BoomerAMGSetAggNumLevels", _i, [_p, _i]),
    ("HYPRE_BoomerAMGSetNumPaths", _i, [_p, _i]),
    ("HYPRE_BoomerAMGSetAggInterpType", _i, [_p, _i]),
    ("HYPRE_BoomerAMGSetAggTruncFactor", _i, [_p, _d]),
    ("HYPRE_BoomerAMGSetAggP12TruncFactor", _i, [_p, _d]),
    ("HYPRE_BoomerAMGSetAggPMaxElmts", _i, [_p, _i]),
    ("HYPRE_BoomerAMGSetAggP12MaxElmts", _i, [_p, _i]),
    ("HYPRE_BoomerAMGSetInterpType", _i, [_p, _i]),
    ("HYPRE_BoomerAMGSetSepWeight", _i, [_p, _i]),
    ("HYPRE_BoomerAMGSetSeqThreshold", _i, [_p, _i]),
    ("HYPRE_BoomerAMGSetNumFunctions", _i, [_p, _i]),
    ("HYPRE_BoomerAMGSetRedundant", _i, [_p, _i]),
    ("HYPRE_BoomerAMGSetTruncFactor", _i, [_p, _d]),
    ("HYPRE_BoomerAMGSetPMaxElmts", _i, [_p, _i]),
    ("HYPRE_BoomerAMGSetCycleType", _i, [_p, _i]),
    ("HYPRE_BoomerAMGSetNumSweeps", _i, [_p, _i]),
    ("HYPRE_BoomerAMGSetCycleNumSweeps", _i, [_p, _i, _i]),
    ("HYPRE_BoomerAMGSetRelaxType", _i, [_p, _i]),
    ("HYPRE_BoomerAMGSetCycleRelaxType", _i, [_p, _i, _i]),
    ("HYPRE_BoomerAMGSetRelaxOrder", _i, [_p, _i]),
    ("HYPRE_BoomerAMGSetRelaxWt", _i, [_p, _d]),
    ("HYPRE_BoomerAMGSetOuterWt", _i, [_p, _d]),
    ("HYPRE_BoomerAMGSetLevelRelaxWt", _i, [_p, _d, _i]),
    ("HYPRE_BoomerAMGSetLevelOuterWt", _i, [_p, _d, _i]),
    ("hypreve_BoomerAMGGetLevelWeights", _i, [_p, _i, _pd, _pd]),
    ("HYPRE_BoomerAMGSetChebyOrder", _i, [_p, _i]),
    ("HYPRE_BoomerAMGSetChebyFraction", _i, [_p, _d]),
    ("HYPRE_BoomerAMGSetChebyScale", _i, [_p, _i]),
    ("HYPRE_BoomerAMGSetChebyVariant", _i, [_p, _i]),
    ("HYPRE_BoomerAMGSetChebyEigEst", _i, [_p, _i]),
    ("hypreve_BoomerAMGGetChebyInfo", _i, [_p, _i, C.POINTER(_i), C.POINTER(_d), C.POINTER(_d), C.POINTER(_i)]),
    ("HYPRE_BoomerAMGSetPrintLevel", _i, [_p, _i]),
    ("HYPRE_BoomerAMGSetLogging", _i, [_p, _i]),
    ("HYPRE_BoomerAMGGetNumLevels", _i, [_p, _pi]),
    ("HYPRE_ParCSRPCGCreate", _i, [_p, C.POINTER(_p)]),
    ("HYPRE_ParCSRPCGDestroy", _i, [_p]),
    ("HYPRE_ParCSRPCGSetup", _i, [_p, _p, _p, _p]),
    ("HYPRE_ParCSRPCGSolve", _i, [_p, _p, _p, _p]),
    ("HYPRE_ParCSRPCGSetTol", _i, [_p, _d]),
    ("HYPRE_ParCSRPCGSetMaxIter", _i, [_p, _i]),
    ("HYPRE_ParCSRPCGSetTwoNorm", _i, [_p, _i]),
    ("HYPRE_ParCSRPCGSetPrecond", _i, [_p, _p, _p, _p]),
    ("HYPRE_ParCSRPCGSetPrintLevel", _i, [_p, _i]),
    ("HYPRE_ParCSRPCGGetNumIterations", _i, [_p, _pi]),
    ("HYPRE_ParCSRPCGGetFinalRelativeResidualNorm", _i, [_p, _pd]),
    ("hypreve_CommGetUniqueId", _i, [_p]),
    ("hypreve_CommCreate", _i, [_i, _i, _p, C.POINTER(_p)]),
    ("hypreve_CommDestroy", _i, [_p]),
    ("hypreve_CommSelfTest", _i, [_p]),
    ("hypreve_CommCreateLoopback", _i, [_i, C.POINTER(_p)]),
    ("hypreve_CommCreateShm", _i, [_i, _i, C.c_char_p, C.POINTER(_p)]),
    ("hypreve_ParCSRMatrixCreateFromCSR", _i, [_p, _i, _i, _i, _pi, _pi, _pd, C.POINTER(_p)]),
    ("hypreve_ParVectorDeviceData", _p, [_p]),
    ("hypreve_ParVectorLocalSize", _i, [_p]),
    ("hypreve_ParVectorCopyToHost", _i, [_p, _pd]),
    ("hypreve_ParVectorCopyFromHost", _i, [_p, _pd]),
    ("hypreve_ParVectorSetRandomValues", _i, [_p, _i]),
    ("hypreve_BoomerAMGSetNumBlocks", _i, [_p, _i]),
    ("hypreve_BoomerAMGSetBlockBands", _i, [_p, _i, _i]),
    ("hypreve_BoomerAMGSetUseGraph", _i, [_p, _i]),
    ("hypreve_BoomerAMGSetSellPolicy", _i, [_p, _i]),
    ("hypreve_BoomerAMGSetAggloRows", _i, [_p, _i]),
    ("hypreve_BoomerAMGGetComplexities", _i, [_p, _pd, _pd, _pd]),
    ("hypreve_BoomerAMGGetLevelInfo", _i, [_p, _i, _pi, _pi64, _pi64]),
    ("hypreve_BoomerAMGGetLevelMatrix", _i, [_p, _i, _i, _pi, _pi, _pi64, _pi, _pi, _pd]),
    ("hypreve_BoomerAMGGetLevelVector", _i, [_p, _i, _i, _pi, _p]),
    ("hypreve_BoomerAMGGetCoarseMatrix", _i, [_p, _pi, _pd]),
    ("hypreve_BoomerAMGGetRelaxInfo", _i, [_p, _pi, _pi, _pd, _pi]),
    ("hypreve_BoomerAMGSetupHost", _i, [_p, _p]),
    ("hypreve_BoomerAMGPartitionCheck", _i, [_p, _i]),
    ("hypreve_BoomerAMGDistSetupCheck", _i, [_p, _p, _i]),
    ("hypreve_BoomerAMGCycle", _i, [_p, _p, _p]),
    ("hypreve_BoomerAMGGetKernelStats", _i, [_p, _pd, _i]),
    ("hypreve_BenchFineSpMV", _i, [_p, _i, _pd, _pd]),
    ("hypreve_BenchFineSpMVStoredBytes", _i, [_p, _pd]),
    ("hypreve_BoomerAMGGetLevelLayout", _i, [_p, _i, _i, _pi]),
    ("hypreve_BoomerAMGSetGsRankStarts", _i, [_p, _i, _pi]),
    ("hypreve_BoomerAMGSetRankEmulation", _i, [_p, _i, _pi]),
    ("HYPRE_BoomerAMGSetDofFunc", _i, [_p, _pi]),
    ("hypreve_BoomerAMGSetCoarsenRankStarts", _i, [_p, _i, _pi]),
    ("hypreve_BoomerAMGGsScheduleCheck", _i, [_p, _i]),
    ("hypreve_BoomerAMGGsScheduleStats", _i, [_p, _i, _i, _i, _pi64]),
    ("hypreve_BoomerAMGGetCycleCommStats", _i, [_p, _i, _pi64]),
    ("hypreve_BoomerAMGStencilLayoutCheck", _i, [_p, _i, _pi, _pi]),
    ("hypreve_GridStencilAddressable", _i, [_i, _i, _i]),
    ("hypreve_BoomerAMGCodedLayoutCheck", _i, [_p, _i, _i, _pi, _pi]),
    ("hypreve_SetKnob", _i, [_i, _i]),
    ("hypreve_BoomerAMGSetDeviceSetup", _i, [_p, _i]),
    ("hypreve_BoomerAMGGetSetupLog", _i, [_p, C.c_char_p, _i]),
    ("hypreve_BoomerAMGGetSetupPath", _i, [_p, C.POINTER(C.c_int)]),
    ("hypreve_BenchLevelOp", _i, [_p, _i, _i, _i, _pd, _pd, _pd]),
    ("hypreve_BenchLevelOpStoredBytes", _i, [_p, _i, _i, _pd]),
    ("hypreve_BenchOperator", _i, [_p, _i, _i, _i, _i, _pd, _pd, C.c_char_p, _i]),
    ("hypreve_BenchStream", _i, [_i, C.c_int64, _i, _pd]),
    ("hypreve_DeviceSynchronize", _i, []),
    ("hypreve_BuildInfo", C.c_char_p, []),
    ("hypreve_LastErrorMessage", C.c_char_p, []),
]


def _declare(L):
    for name, res, args in SIGNATURES:
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args


class HypreError(RuntimeError):
    pass


def check(rc: int, what: str = ""):
    if rc:
        msg = lib().hypreve_LastErrorMessage().decode()
        lib().HYPRE_ClearAllErrors()
        raise HypreError(f"{what} failed (hypre error {rc}): {msg}")


def _ptr(a, ct):
    return a.ctypes.data_as(C.POINTER(ct))


class Comm:
    """Communicator over RCCL: one process per GPU (hypreve_CommCreate).  The
    128-byte unique id comes from rank 0 (Comm.unique_id) and is broadcast by
    the caller's own launcher (torch.distributed, MPI_Bcast, ...)."""

    def __init__(self, h, rank, size):
        self.h, self.rank, self.size = h, rank, size

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        check(lib().hypreve_CommGetUniqueId(buf), "CommGetUniqueId")
        return buf.raw

    @classmethod
    def create(cls, rank, size, uid: bytes):
        assert len(uid) == 128
        h = _p()
        buf = C.create_string_buffer(uid, 128)
        check(lib().hypreve_CommCreate(rank, size, buf, C.byref(h)), "CommCreate")
        return cls(h, rank, size)

    @classmethod
    def loopback(cls, size):
        """`size` virtual ranks on this process's GPU; drive each from its own thread."""
        hs = (_p * size)()
        check(lib().hypreve_CommCreateLoopback(size, hs), "CommCreateLoopback")
        return [cls(_p(hs[r]), r, size) for r in range(size)]

    @classmethod
    def shm(cls, rank, size, name: str):
        """One process of `size` on this host over the shared-memory segment
        `name` (host-staged; several processes may share one GPU)."""
        h = _p()
        check(lib().hypreve_CommCreateShm(rank, size, name.encode(), C.byref(h)), "CommCreateShm")
        return cls(h, rank, size)

    def self_test(self):
        """Collective transport check (exchange incl. self, all-reduce,
        all-gather, broadcast); raises on a mismatch."""
        check(lib().hypreve_CommSelfTest(self.h), "CommSelfTest")

    def destroy(self):
        if self.h:
            lib().hypreve_CommDestroy(self.h)
            self.h = None


# ---------------------------------------------------------------------------
# thin object layer
# ---------------------------------------------------------------------------
class ParCSRMatrix:
    def __init__(self, handle, n):
        self.h = handle
        self.n = n

    @classmethod
    def laplacian(cls, nx, ny, nz, cx=1.0, cy=1.0, cz=1.0, comm=None, P=1, Q=1, R=1, p=0, q=0, r=0):
        """GenerateLaplacian as test/ij.c:7790 BuildParLaplacian calls it.  With a
        Comm, this rank builds its block (p, q, r) of the P x Q x R processor grid."""
        v0 = (2.0 * cx if nx > 1 else 0.0) + (2.0 * cy if ny > 1 else 0.0) + (2.0 * cz if nz > 1 else 0.0)
        vals = np.array([v0, -cx, -cy, -cz], dtype=np.float64)
        h = lib().GenerateLaplacian(comm.h if comm else None, nx, ny, nz, P, Q, R, p, q, r, _ptr(vals, C.c_double))
        if not h:
            check(lib().HYPRE_GetError() or 1, "GenerateLaplacian")
        M = cls(h, nx * ny * nz)
        M.first, last = M.local_range()
        M.n = last - M.first + 1
        M.global_n = nx * ny * nz
        return M

    def local_range(self):
        """(first_row, last_row) owned by this rank (HYPRE_ParCSRMatrixGetLocalRange)."""
        r0, r1, c0, c1 = (C.c_int() for _ in range(4))
        check(lib().HYPRE_ParCSRMatrixGetLocalRange(self.h, C.byref(r0), C.byref(r1), C.byref(c0), C.byref(c1)),
              "GetLocalRange")
        return r0.value, r1.value

    @classmethod
    def laplacian27(cls, nx, ny, nz, comm=None, P=1, Q=1, R=1, p=0, q=0, r=0):
        """GenerateLaplacian27pt (diagonal 26, neighbours -1); with a Comm this
        rank's block (p, q, r) of the P x Q x R processor grid."""
        vals = np.array([26.0, -1.0], dtype=np.float64)
        h = lib().GenerateLaplacian27pt(comm.h if comm else None, nx, ny, nz, P, Q, R, p, q, r,
                                        _ptr(vals, C.c_double))
        if not h:
            check(lib().HYPRE_GetError() or 1, "GenerateLaplacian27pt")
        M = cls(h, nx * ny * nz)
        M.first, last = M.local_range()
        M.n = last - M.first + 1
        M.global_n = nx * ny * nz
        return M

    @classmethod
    def from_scipy(cls, A):
        A = A.tocsr()
        n = A.shape[0]
        ip = np.ascontiguousarray(A.indptr, dtype=np.int32)
        jj = np.ascontiguousarray(A.indices, dtype=np.int32)
        vv = np.ascontiguousarray(A.data, dtype=np.float64)
        h = _p()
        check(lib().hypreve_ParCSRMatrixCreateFromCSR(None, 0, n, n, _ptr(ip, C.c_int), _ptr(jj, C.c_int),
                                                      _ptr(vv, C.c_double), C.byref(h)), "CreateFromCSR")
        return cls(h, n)

    def bench_operator(self, op=0, policy=0, nbands=8, reps=20):
        """(avg ms, stored bytes, layout text) of op applied to this matrix
        alone (hypreve_BenchOperator; tuning)."""
        ms, by = C.c_double(), C.c_double()
        buf = C.create_string_buffer(160)
        check(lib().hypreve_BenchOperator(self.h, op, policy, nbands, reps, C.byref(ms), C.byref(by), buf, 160),
              "BenchOperator")
        return ms.value, by.value, buf.value.decode()

    def matvec(self, alpha, x, beta, y):
        check(lib().HYPRE_ParCSRMatrixMatvec(alpha, self.h, x.h, beta, y.h), "Matvec")

    def destroy(self):
        if self.h:
            lib().HYPRE_ParCSRMatrixDestroy(self.h)
            self.h = None


class ParVector:
    def __init__(self, n, data=None, comm=None, first=0, global_n=None):
        """n owned entries starting at global index first (HYPRE_ParVectorCreate)."""
        self.n = n
        h = _p()
        part = np.array([first, first + n], dtype=np.int32)
        gn = n if global_n is None else global_n
        check(lib().HYPRE_ParVectorCreate(comm.h if comm else None, gn, _ptr(part, C.c_int), C.byref(h)),
              "ParVectorCreate")
        self.h = h
        check(lib().HYPRE_ParVectorInitialize(h), "ParVectorInitialize")
        if data is not None:
            self.set(data)

    def set(self, data):
        a = np.ascontiguousarray(data, dtype=np.float64)
        assert a.size == self.n
        check(lib().hypreve_ParVectorCopyFromHost(self.h, _ptr(a, C.c_double)), "CopyFromHost")

    def get(self):
        out = np.empty(self.n, dtype=np.float64)
        check(lib().hypreve_ParVectorCopyToHost(self.h, _ptr(out, C.c_double)), "CopyToHost")
        return out

    def fill(self, v):
        check(lib().HYPRE_ParVectorSetConstantValues(self.h, v), "SetConstantValues")

    def dot(self, other):
        r = C.c_double()
        check(lib().HYPRE_ParVectorInnerProd(self.h, other.h, C.byref(r)), "InnerProd")
        return r.value

    def destroy(self):
        if self.h:
            lib().HYPRE_ParVectorDestroy(self.h)
            self.h = None


class BoomerAMG:
    """HYPRE_BoomerAMG* with keyword settings named like the Set* calls."""

    _setters = {
        "tol": ("HYPRE_BoomerAMGSetTol", float), "max_iter": ("HYPRE_BoomerAMGSetMaxIter", int),
        "min_iter": ("HYPRE_BoomerAMGSetMinIter", int),
        "max_coarse_size": ("HYPRE_BoomerAMGSetMaxCoarseSize", int),
        "min_coarse_size": ("HYPRE_BoomerAMGSetMinCoarseSize", int),
        "max_levels": ("HYPRE_BoomerAMGSetMaxLevels", int),
        "strong_threshold": ("HYPRE_BoomerAMGSetStrongThreshold", float),
        "max_row_sum": ("HYPRE_BoomerAMGSetMaxRowSum", float),
        "coarsen_type": ("HYPRE_BoomerAMGSetCoarsenType", int),
        "interp_type": ("HYPRE_BoomerAMGSetInterpType", int),
        "sep_weight": ("HYPRE_BoomerAMGSetSepWeight", int),
        "seq_threshold": ("HYPRE_BoomerAMGSetSeqThreshold", int),
        "num_functions": ("HYPRE_BoomerAMGSetNumFunctions", int),
        "redundant": ("HYPRE_BoomerAMGSetRedundant", int),
        "trunc_factor": ("HYPRE_BoomerAMGSetTruncFactor", float),
        "P_max_elmts": ("HYPRE_BoomerAMGSetPMaxElmts", int),
        "cycle_type": ("HYPRE_BoomerAMGSetCycleType", int),
        "num_sweeps": ("HYPRE_BoomerAMGSetNumSweeps", int),
        "relax_type": ("HYPRE_BoomerAMGSetRelaxType", int),
        "relax_order": ("HYPRE_BoomerAMGSetRelaxOrder", int),
        "relax_wt": ("HYPRE_BoomerAMGSetRelaxWt", float), "outer_wt": ("HYPRE_BoomerAMGSetOuterWt", float),
        "print_level": ("HYPRE_BoomerAMGSetPrintLevel", int), "converge_type": ("HYPRE_BoomerAMGSetConvergeType", int),
        "num_blocks": ("hypreve_BoomerAMGSetNumBlocks", int), "use_graph": ("hypreve_BoomerAMGSetUseGraph", int),
        "sell_policy": ("hypreve_BoomerAMGSetSellPolicy", int),
        "device_setup": ("hypreve_BoomerAMGSetDeviceSetup", int),
        "agglo_rows": ("hypreve_BoomerAMGSetAggloRows", int),
        "agg_num_levels": ("HYPRE_BoomerAMGSetAggNumLevels", int), "num_paths": ("HYPRE_BoomerAMGSetNumPaths", int),
        "agg_interp_type": ("HYPRE_BoomerAMGSetAggInterpType", int),
        "agg_trunc_factor": ("HYPRE_BoomerAMGSetAggTruncFactor", float),
        "agg_P_max_elmts": ("HYPRE_BoomerAMGSetAggPMaxElmts", int),
        "agg_P12_trunc_factor": ("HYPRE_BoomerAMGSetAggP12TruncFactor", float),
        "agg_P12_max_elmts": ("HYPRE_BoomerAMGSetAggP12MaxElmts", int),
        "measure_type": ("HYPRE_BoomerAMGSetMeasureType", int),
        "cheby_order": ("HYPRE_BoomerAMGSetChebyOrder", int), "cheby_fraction": ("HYPRE_BoomerAMGSetChebyFraction", float),
        "cheby_scale": ("HYPRE_BoomerAMGSetChebyScale", int), "cheby_variant": ("HYPRE_BoomerAMGSetChebyVariant", int),
        "cheby_eig_est": ("HYPRE_BoomerAMGSetChebyEigEst", int),
    }

    def __init__(self, **kw):
        h = _p()
        check(lib().HYPRE_BoomerAMGCreate(C.byref(h)), "BoomerAMGCreate")
        self.h = h
        self.set(**kw)

    def set(self, **kw):
        for k, v in kw.items():
            if k == "cycle_relax_type":
                for kk, t in v.items():
                    check(lib().HYPRE_BoomerAMGSetCycleRelaxType(self.h, int(t), int(kk)), k)
                continue
            if k in ("level_relax_wt", "level_outer_wt"):  # (weight, level), ij -wl / -owl
                fn = "HYPRE_BoomerAMGSetLevelRelaxWt" if k == "level_relax_wt" else "HYPRE_BoomerAMGSetLevelOuterWt"
                check(getattr(lib(), fn)(self.h, float(v[0]), int(v[1])), fn)
                continue
            if k == "cycle_num_sweeps":
                for kk, t in v.items():
                    check(lib().HYPRE_BoomerAMGSetCycleNumSweeps(self.h, int(t), int(kk)), k)
                continue
            fn, ty = self._setters[k]
            check(getattr(lib(), fn)(self.h, ty(v)), fn)

    def setup(self, A, b=None, x=None):
        check(lib().HYPRE_BoomerAMGSetup(self.h, A.h, b.h if b else None, x.h if x else None), "BoomerAMGSetup")

    def partition_check(self, size):
        check(lib().hypreve_BoomerAMGPartitionCheck(self.h, size), "PartitionCheck")

    def dist_setup_check(self, A, size):
        check(lib().hypreve_BoomerAMGDistSetupCheck(self.h, A.h, size), "DistSetupCheck")

    def setup_host(self, A):
        check(lib().hypreve_BoomerAMGSetupHost(self.h, A.h), "BoomerAMGSetupHost")

    def solve(self, A, b, x, allow_conv_error=True):
        rc = lib().HYPRE_BoomerAMGSolve(self.h, A.h, b.h, x.h)
        if rc and not (allow_conv_error and rc == HYPRE_ERROR_CONV):
            check(rc, "BoomerAMGSolve")
        lib().HYPRE_ClearAllErrors()
        return self.num_iterations(), self.final_rel_res()

    def cycle(self, f, u):
        check(lib().hypreve_BoomerAMGCycle(self.h, f.h, u.h), "BoomerAMGCycle")

    def num_iterations(self):
        v = C.c_int()
        lib().HYPRE_BoomerAMGGetNumIterations(self.h, C.byref(v))
        return v.value

    def final_rel_res(self):
        v = C.c_double()
        lib().HYPRE_BoomerAMGGetFinalRelativeResidualNorm(self.h, C.byref(v))
        return v.value

    def num_levels(self):
        v = C.c_int()
        lib().HYPRE_BoomerAMGGetNumLevels(self.h, C.byref(v))
        return v.value

    def complexities(self):
        g, o, c = C.c_double(), C.c_double(), C.c_double()
        lib().hypreve_BoomerAMGGetComplexities(self.h, C.byref(g), C.byref(o), C.byref(c))
        return g.value, o.value, c.value

    def level_info(self, l):
        r, a, p = C.c_int(), C.c_int64(), C.c_int64()
        check(lib().hypreve_BoomerAMGGetLevelInfo(self.h, l, C.byref(r), C.byref(a), C.byref(p)), "GetLevelInfo")
        return r.value, a.value, p.value

    def level_matrix(self, l, which=0):
        """(indptr, indices, data, shape) of A_l (which=0), P_l (1) or R_l = P_l^T (2)."""
        nr, nc, nz = C.c_int(), C.c_int(), C.c_int64()
        L = lib()
        check(L.hypreve_BoomerAMGGetLevelMatrix(self.h, l, which, C.byref(nr), C.byref(nc), C.byref(nz),
                                                None, None, None), "GetLevelMatrix")
        ip = np.zeros(nr.value + 1, dtype=np.int32)
        jj = np.zeros(max(1, nz.value), dtype=np.int32)
        vv = np.zeros(max(1, nz.value), dtype=np.float64)
        check(L.hypreve_BoomerAMGGetLevelMatrix(self.h, l, which, None, None, None, _ptr(ip, C.c_int),
                                                _ptr(jj, C.c_int), _ptr(vv, C.c_double)), "GetLevelMatrix")
        return ip, jj[: nz.value], vv[: nz.value], (nr.value, nc.value)

    def level_vector(self, l, which):
        n = C.c_int()
        check(lib().hypreve_BoomerAMGGetLevelVector(self.h, l, which, C.byref(n), None), "GetLevelVector")
        # 0 cf, 1 l1, 2 Chebyshev ds, 3 hybrid-GS block starts (N-rank emulation)
        out = np.zeros(n.value, dtype=np.int32 if which in (0, 3) else np.float64)
        if n.value:
            lib().hypreve_BoomerAMGGetLevelVector(self.h, l, which, None, out.ctypes.data_as(C.c_void_p))
        return out

    def cheby_info(self, l):
        """(coefficients, (max_eig, min_eig), (order, scale, variant)) of level l's Chebyshev smoother."""
        n = C.c_int()
        co = (C.c_double * 5)()
        eig = (C.c_double * 2)()
        prm = (C.c_int * 3)()
        check(lib().hypreve_BoomerAMGGetChebyInfo(self.h, l, C.byref(n), co, eig, prm), "GetChebyInfo")
        return np.array(co[: n.value]), (eig[0], eig[1]), (prm[0], prm[1], prm[2])

    def coarse_matrix(self):
        n = C.c_int()
        lib().hypreve_BoomerAMGGetCoarseMatrix(self.h, C.byref(n), None)
        out = np.zeros(n.value * n.value, dtype=np.float64)
        if n.value:
            lib().hypreve_BoomerAMGGetCoarseMatrix(self.h, None, _ptr(out, C.c_double))
        return out.reshape(n.value, n.value) if n.value else out

    def relax_info(self):
        rt = np.zeros(4, dtype=np.int32)
        ns = np.zeros(4, dtype=np.int32)
        w = np.zeros(2, dtype=np.float64)
        misc = np.zeros(4, dtype=np.int32)
        lib().hypreve_BoomerAMGGetRelaxInfo(self.h, _ptr(rt, C.c_int), _ptr(ns, C.c_int), _ptr(w, C.c_double),
                                            _ptr(misc, C.c_int))
        return dict(relax_type=rt.tolist(), num_sweeps=ns.tolist(), relax_weight=float(w[0]), omega=float(w[1]),
                    relax_order=int(misc[0]), cycle_type=int(misc[1]), num_blocks=int(misc[2]),
                    user_relax_type=int(misc[3]))

    def level_weights(self, level):
        """(relax_weight, omega) the cycle uses on level."""
        w, o = C.c_double(), C.c_double()
        check(lib().hypreve_BoomerAMGGetLevelWeights(self.h, level, C.byref(w), C.byref(o)), "GetLevelWeights")
        return w.value, o.value

    def gs_schedule_check(self, num_blocks):
        check(lib().hypreve_BoomerAMGGsScheduleCheck(self.h, num_blocks), "GsScheduleCheck")

    def cycle_comm_stats(self):
        """This rank's communication in one V-cycle, per level: halo exchanges,
        bytes sent, all-gathers, all-gather bytes, all-reduces."""
        out = []
        for l in range(self.num_levels()):
            v = (C.c_int64 * 5)()
            check(lib().hypreve_BoomerAMGGetCycleCommStats(self.h, l, v), "GetCycleCommStats")
            out.append(dict(zip(("exchanges", "bytes", "allgathers", "allgather_bytes", "allreduces"), list(v))))
        return out

    def gs_schedule_stats(self, level, forward, num_blocks):
        """Packed hybrid-GS schedule of level `level`: nnz, stored entries,
        steps, teams, longest team (steps), blocks."""
        out = (C.c_int64 * 6)()
        check(lib().hypreve_BoomerAMGGsScheduleStats(self.h, level, int(forward), num_blocks, out),
              "GsScheduleStats")
        return dict(zip(("nnz", "entries", "steps", "teams", "max_steps", "blocks"), list(out)))

    def stencil_layout_check(self, level=0):
        """(slots per pattern, patterns) of level's A in the stencil layout,
        checked row by row against the CSR on the host; (0, 0) when the
        operator is not a constant-coefficient stencil."""
        w, npat = C.c_int(), C.c_int()
        check(lib().hypreve_BoomerAMGStencilLayoutCheck(self.h, level, C.byref(w), C.byref(npat)), "StencilLayoutCheck")
        return w.value, npat.value

    SETUP_PATHS = ("one process", "one process, rank emulation", "distributed", "gathered, rank emulation",
                   "gathered, one process")

    def setup_path(self):
        """The path the last setup took (hypreve_BoomerAMGGetSetupPath), by name."""
        v = C.c_int()
        check(lib().hypreve_BoomerAMGGetSetupPath(self.h, C.byref(v)), "GetSetupPath")
        return self.SETUP_PATHS[v.value] if v.value >= 0 else None

    def setup_log(self):
        """The setup's log: levels, phase times, rows the device setup left to the host."""
        buf = C.create_string_buffer(1 << 16)
        check(lib().hypreve_BoomerAMGGetSetupLog(self.h, buf, 1 << 16), "GetSetupLog")
        return buf.value.decode()

    def coded_layout_check(self, level=0, which=1):
        """(distinct offsets, distinct values) of level's P (which 1) or R (2)
        in the offset-coded layout, checked row by row against the CSR on the
        host; (0, 0) when the operator does not code in 16 bits."""
        no, nv = C.c_int(), C.c_int()
        check(lib().hypreve_BoomerAMGCodedLayoutCheck(self.h, level, which, C.byref(no), C.byref(nv)),
              "CodedLayoutCheck")
        return no.value, nv.value

    def bench_level_op(self, level, which=0, reps=20):
        """(avg_ms, algorithmic bytes, padded entries) of A_l (0), P_l (1) or R_l (2)."""
        ms, by, pz = C.c_double(), C.c_double(), C.c_double()
        check(lib().hypreve_BenchLevelOp(self.h, level, which, reps, C.byref(ms), C.byref(by), C.byref(pz)),
              "BenchLevelOp")
        return ms.value, by.value, pz.value

    def set_block_bands(self, nbands, which="APR"):
        """Re-key the row-block traversal of the A / P / R operators (0 bands =
        natural order); tuning only."""
        mask = (1 if "A" in which else 0) | (2 if "P" in which else 0) | (4 if "R" in which else 0)
        check(lib().hypreve_BoomerAMGSetBlockBands(self.h, int(nbands), mask), "SetBlockBands")

    def level_op_stored_bytes(self, level, which=0):
        """Bytes one bench_level_op launch streams in the stored layout (+ vectors)."""
        by = C.c_double()
        check(lib().hypreve_BenchLevelOpStoredBytes(self.h, level, which, C.byref(by)), "BenchLevelOpStoredBytes")
        return by.value

    def bench_fine_spmv(self, reps=20):
        ms, by = C.c_double(), C.c_double()
        check(lib().hypreve_BenchFineSpMV(self.h, reps, C.byref(ms), C.byref(by)), "BenchFineSpMV")
        return ms.value, by.value

    def set_gs_rank_starts(self, starts):
        """Hybrid GS with the row blocks of an N-rank run (level-0 starts, N+1
        entries); None clears it.  Takes effect at setup."""
        if starts is None or len(starts) <= 2:
            check(lib().hypreve_BoomerAMGSetGsRankStarts(self.h, 0, None), "SetGsRankStarts")
            return
        arr = (C.c_int * len(starts))(*[int(v) for v in starts])
        check(lib().hypreve_BoomerAMGSetGsRankStarts(self.h, len(starts) - 1, arr), "SetGsRankStarts")

    def set_dof_func(self, dof):
        """The function of every row (HYPRE_BoomerAMGSetDofFunc); the array is
        kept alive here and read at Setup.  None clears it."""
        if dof is None:
            self._dof = None
            check(lib().HYPRE_BoomerAMGSetDofFunc(self.h, None), "SetDofFunc")
            return
        self._dof = (C.c_int * len(dof))(*[int(v) for v in dof])
        check(lib().HYPRE_BoomerAMGSetDofFunc(self.h, self._dof), "SetDofFunc")

    def set_rank_emulation(self, starts):
        """Reproduce a reference N-rank setup in one process (level-0 row starts,
        N+1 entries; hypreve_BoomerAMGSetRankEmulation); None clears it."""
        if starts is None or len(starts) <= 2:
            check(lib().hypreve_BoomerAMGSetRankEmulation(self.h, 0, None), "SetRankEmulation")
            return
        arr = (C.c_int * len(starts))(*[int(v) for v in starts])
        check(lib().hypreve_BoomerAMGSetRankEmulation(self.h, len(starts) - 1, arr), "SetRankEmulation")

    def set_coarsen_rank_starts(self, starts):
        """HMIS coarsened as an N-rank run's distributed setup does it (level-0
        row starts, N+1 entries; hypreve_BoomerAMGSetCoarsenRankStarts), the
        rest of the setup one-process; None clears it.  Takes effect at setup."""
        if starts is None or len(starts) <= 2:
            check(lib().hypreve_BoomerAMGSetCoarsenRankStarts(self.h, 0, None), "SetCoarsenRankStarts")
            return
        arr = (C.c_int * len(starts))(*[int(v) for v in starts])
        check(lib().hypreve_BoomerAMGSetCoarsenRankStarts(self.h, len(starts) - 1, arr), "SetCoarsenRankStarts")

    LAYOUTS = ("padded", "jagged", "wide", "jag-pw", "dict", "delta", "delta+vt8", "delta+vt16", "padded+vt16",
               "jagged+vt16", "dict-ranges", "stencil", "coded", "packed", "grid-stencil", "dict-wide", "coded-jag")

    def level_layout(self, level, which=0):
        """Device layout name of A_l (0), P_l (1) or R_l (2) (interior rows)."""
        k = C.c_int()
        check(lib().hypreve_BoomerAMGGetLevelLayout(self.h, level, which, C.byref(k)), "GetLevelLayout")
        return self.LAYOUTS[k.value]

    def fine_spmv_stored_bytes(self):
        """Bytes the finest SpMV streams in its stored layout (+ vectors)."""
        by = C.c_double()
        check(lib().hypreve_BenchFineSpMVStoredBytes(self.h, C.byref(by)), "BenchFineSpMVStoredBytes")
        return by.value

    def destroy(self):
        if self.h:
            lib().HYPRE_BoomerAMGDestroy(self.h)
            self.h = None


class PCG:
    def __init__(self, tol=1e-8, max_iter=1000, two_norm=1, print_level=0):
        h = _p()
        check(lib().HYPRE_ParCSRPCGCreate(None, C.byref(h)), "PCGCreate")
        self.h = h
        lib().HYPRE_ParCSRPCGSetTol(h, tol)
        lib().HYPRE_ParCSRPCGSetMaxIter(h, max_iter)
        lib().HYPRE_ParCSRPCGSetTwoNorm(h, two_norm)
        lib().HYPRE_ParCSRPCGSetPrintLevel(h, print_level)
        self.precond = None

    def set(self, tol=None, max_iter=None):
        if tol is not None:
            check(lib().HYPRE_ParCSRPCGSetTol(self.h, float(tol)), "PCGSetTol")
        if max_iter is not None:
            check(lib().HYPRE_ParCSRPCGSetMaxIter(self.h, int(max_iter)), "PCGSetMaxIter")

    def set_precond_amg(self, amg: BoomerAMG, setup=True):
        """BoomerAMG as the preconditioner; setup=False: PCGSetup leaves an
        already set-up hierarchy as it is (no precond_setup function)."""
        L = lib()
        solve = C.cast(L.HYPRE_BoomerAMGSolve, C.c_void_p)
        setup = C.cast(L.HYPRE_BoomerAMGSetup, C.c_void_p) if setup else None
        check(L.HYPRE_ParCSRPCGSetPrecond(self.h, solve, setup, amg.h), "PCGSetPrecond")
        self.precond = amg

    def setup(self, A, b, x):
        check(lib().HYPRE_ParCSRPCGSetup(self.h, A.h, b.h, x.h), "PCGSetup")

    def solve(self, A, b, x, allow_conv_error=True):
        rc = lib().HYPRE_ParCSRPCGSolve(self.h, A.h, b.h, x.h)
        if rc and not (allow_conv_error and rc == HYPRE_ERROR_CONV):
            check(rc, "PCGSolve")
        lib().HYPRE_ClearAllErrors()
        it, r = C.c_int(), C.c_double()
        lib().HYPRE_ParCSRPCGGetNumIterations(self.h, C.byref(it))
        lib().HYPRE_ParCSRPCGGetFinalRelativeResidualNorm(self.h, C.byref(r))
        return it.value, r.value

    def destroy(self):
        if self.h:
            lib().HYPRE_ParCSRPCGDestroy(self.h)
            self.h = None


def init():
    check(lib().HYPRE_Init(), "HYPRE_Init")


def bench_stream(elem_bytes, n, reps=20):
    """Average ms of a read-only stream over n elements of elem_bytes (2, 4, 8 or 16),
    or (elem_bytes -1 / -2 / -5) of a read/write mix: that many n-double streams
    read and one written."""
    ms = C.c_double()
    check(lib().hypreve_BenchStream(elem_bytes, n, reps, C.byref(ms)), "BenchStream")
    return ms.value


def ij_amg_defaults(solver_id=0):
    """BoomerAMG settings test/ij.c applies before its command-line options
    (ij.c:1181-1199, 3365-3540): max_row_sum 1.0, tol 1e-8 (solver 0),
    P_max_elmts 4, coarsen HMIS (10), ext+i (6), print level 3."""
    return dict(max_row_sum=1.0, tol=1e-8 if solver_id == 0 else 0.0, max_iter=100 if solver_id == 0 else 1,
                strong_threshold=0.25, trunc_factor=0.0, P_max_elmts=4, max_coarse_size=9, max_levels=25,
                cycle_type=1, relax_wt=1.0, outer_wt=1.0)


def set_knob(knob_id, value):
    """Tuning knob read at kernel launch (hypreve_SetKnob; results unchanged)."""
    check(lib().hypreve_SetKnob(knob_id, value), "SetKnob")
