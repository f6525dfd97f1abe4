"""A plain C program (tests/c_caller/ij_laplace.c) compiled against
include/hypreve.h with gcc -std=c99 -Wall -Wextra -Werror and linked against
libhypreve.so: the header is a C header and the library is callable the way
test/ij.c calls hypre (IJ assembly, BoomerAMG, PCG with BoomerAMGSolve /
BoomerAMGSetup as preconditioner function pointers)."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "c_caller", "ij_laplace.c")
LIBDIR = os.path.join(ROOT, "hypre-ve_amd", "lib")


def _build(tmp_path):
    exe = str(tmp_path / "ij_laplace")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-I" + os.path.join(ROOT, "include"), SRC,
                    "-L" + LIBDIR, "-lhypreve", "-Wl,-rpath," + LIBDIR, "-o", exe], check=True)
    return exe


def _has_gpu():
    try:
        sys.path.insert(0, os.path.join(ROOT, "hypre-ve_amd"))
        import hypreve
        ok = hypreve.lib().HYPRE_Init() == 0
        hypreve.lib().HYPRE_ClearAllErrors()  # the error flag is sticky (hypre_error.c)
        return ok
    except Exception:
        return False


def test_c_caller_builds_and_fails_loudly_without_gpu(tmp_path):
    exe = _build(tmp_path)
    if _has_gpu():
        pytest.skip("a GPU is present (the gpu test runs the program)")
    out = subprocess.run([exe, "6"], capture_output=True, text=True)
    assert out.returncode == 1
    assert "no HIP device" in out.stderr


@pytest.mark.gpu
def test_c_caller_solves(tmp_path, gpu, orc):
    """default.out.0 (TEST_ij/default.saved, -pmis -Pmx 0 -rlx 0 -xisone, 10^3):
    48 iterations to 1e-8; the PCG run takes the oracle's iteration count."""
    exe = _build(tmp_path)
    out = subprocess.run([exe, "10"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    res = {l.split()[0]: (int(l.split()[1]), float(l.split()[2])) for l in out.stdout.splitlines()}
    assert res["amg"][0] == 48 and res["amg"][1] < 1e-8
    hv = gpu
    A = hv.ParCSRMatrix.laplacian(10, 10, 10)
    kw = hv.ij_amg_defaults(1)
    amg = hv.BoomerAMG(**kw)
    amg.setup_host(A)
    O = orc.OracleAMG(amg)
    b = O.matvec(0, 1.0, np.ones(A.n), 0.0, np.zeros(A.n))
    it, rr = O.pcg(b, np.zeros(A.n), 1e-8, 100, 1)
    assert res["pcg"][0] == it
    assert abs(res["pcg"][1] - rr) <= 1e-6 * rr
