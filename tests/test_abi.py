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
