"""The C-ABI library loads on a CPU-only host and exports every symbol that
include/hypreve.h declares (no compute calls here)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "hypreve.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = set()
    for m in re.finditer(r"^\s*(?:HYPRE_Int|HYPRE_ParCSRMatrix|HYPRE_Real\s*\*|const char\s*\*)\s+(\w+)\s*\(", txt, re.M):
        names.add(m.group(1))
    return sorted(names)


def test_header_symbols_exported(hv):
    L = hv.lib()
    syms = header_symbols()
    assert len(syms) > 90
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing


def test_binding_covers_header(hv):
    bound = {n for n, _, _ in hv.SIGNATURES}
    assert set(header_symbols()) <= bound


def test_no_gpu_init_fails_loudly(hv):
    """Without a GPU the solve path refuses to start (no CPU fallback)."""
    if os.path.exists("/dev/kfd"):
        return
    rc = hv.lib().HYPRE_Init()
    assert rc != 0
    hv.lib().HYPRE_ClearAllErrors()


def test_grid_stencil_size_guard(hv):
    """k_grid_stencil's 32-bit buffer byte offsets (kernels.hip, off-grid
    offset 0xFFFFFFF0): DevSell::build_grid takes the grid form only below
    2^29 - 2 points a rank and keeps the per-slice loop above, instead of
    wrapping the offsets and reading zeros."""
    f = hv.lib().hypreve_GridStencilAddressable
    assert f(512, 512, 512) == 1          # the headline grid, one rank
    assert f(512, 512, 2047) == 1         # 2^29 - 2^18 points
    assert f(512, 512, 2048) == 0         # 2^29 points: offsets wrap
    assert f(1024, 1024, 512) == 0
    assert f(64, 8192, 1023) == 1
    assert f(64, 8192, 1024) == 0
    assert f(0, 4, 4) == 0
