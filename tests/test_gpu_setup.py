"""Device setup (hypreve_BoomerAMGSetDeviceSetup, the default of Setup): ext+i
interpolation, its truncation, R = P^T and the Galerkin product RAP on the
GPU (device/setup_dev.hip).  Every level's A, P and R, the CF markers and
the l1 norms must equal the host setup's (hypreve_BoomerAMGSetupHost, the
restatement pinned to the reference's saved runs) byte for byte, including
rows the kernels hand back to the host (tables larger than their LDS)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _hier(hv, amg):
    out = []
    for l in range(amg.num_levels()):
        lev = []
        for w in (0, 1, 2):
            if w and l == amg.num_levels() - 1:
                continue
            ip, jj, vv, shp = amg.level_matrix(l, w)
            lev.append((ip.copy(), jj.copy(), vv.view(np.uint64).copy(), shp))
        lev.append(amg.level_vector(l, 0).copy())
        lev.append(amg.level_vector(l, 1).view(np.uint64).copy() if amg.level_vector(l, 1).size else None)
        out.append(lev)
    return out


def _same(h1, h2):
    assert len(h1) == len(h2)
    for l, (a, b) in enumerate(zip(h1, h2)):
        assert len(a) == len(b), l
        for k, (x, y) in enumerate(zip(a, b)):
            if x is None or y is None:
                assert x is None and y is None, (l, k)
            elif isinstance(x, tuple):
                assert x[3] == y[3], (l, k)
                for u, v in zip(x[:3], y[:3]):
                    assert np.array_equal(u, v), (l, k)
            else:
                assert np.array_equal(x, y), (l, k)


@pytest.mark.parametrize("gen,dims,extra", [
    ("7", (30, 27, 25), {}),
    ("7", (40, 36, 32), {"P_max_elmts": 0}),
    ("7", (24, 22, 20), {"trunc_factor": 0.1, "P_max_elmts": 2}),
    ("7", (28, 26, 24), {"coarsen_type": 10}),
    ("27", (20, 18, 16), {}),
    ("aniso", (28, 26, 24), {}),
    ("aniso", (30, 28, 26), {"agg_num_levels": 1}),
])
def test_device_setup_matches_host(gpu, gen, dims, extra):
    hv = gpu
    if gen == "27":
        A = hv.ParCSRMatrix.laplacian27(*dims)
    elif gen == "aniso":
        A = hv.ParCSRMatrix.laplacian(*dims, cx=0.001, cy=1.0, cz=1.0)
    else:
        A = hv.ParCSRMatrix.laplacian(*dims)
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=18)
    kw.update(extra)
    dev = hv.BoomerAMG(**kw)
    dev.setup(A)
    host = hv.BoomerAMG(**kw)
    host.setup_host(A)
    _same(_hier(hv, dev), _hier(hv, host))
    ctl = hv.BoomerAMG(**kw)
    ctl.set(device_setup=0)
    ctl.setup(A)
    _same(_hier(hv, ctl), _hier(hv, host))
    for s in (dev, host, ctl):
        s.destroy()
    A.destroy()


@pytest.mark.parametrize("gen,dims,extra", [
    ("7", (30, 27, 25), {}),
    ("7", (24, 22, 20), {"coarsen_type": 9}),
    ("27", (20, 18, 16), {"max_row_sum": 0.9}),
    ("aniso", (28, 26, 24), {"strong_threshold": 0.5}),
    ("aniso", (30, 28, 26), {"agg_num_levels": 1}),
    ("7", (48, 44, 40), {}),
])
def test_device_strength_pmis_matches_host(gpu, gen, dims, extra):
    """Strength and PMIS on the device (dev_strength_pmis: one thread a row
    for S, the PMIS passes as kernels over the undecided rows) on every level
    (knob 15 = 1; by default levels of 2^16 rows and more, which the last case
    reaches without it): the hierarchy equals the host setup's byte for byte,
    CF markers included."""
    hv = gpu
    if gen == "27":
        A = hv.ParCSRMatrix.laplacian27(*dims)
    elif gen == "aniso":
        A = hv.ParCSRMatrix.laplacian(*dims, cx=0.001, cy=1.0, cz=1.0)
    else:
        A = hv.ParCSRMatrix.laplacian(*dims)
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=18)
    kw.update(extra)
    host = hv.BoomerAMG(**kw)
    host.setup_host(A)
    big = dims[0] * dims[1] * dims[2] >= 1 << 16
    hv.set_knob(15, 0 if big else 1)
    try:
        dev = hv.BoomerAMG(**kw)
        dev.setup(A)
    finally:
        hv.set_knob(15, 0)
    _same(_hier(hv, dev), _hier(hv, host))
    for s in (dev, host):
        s.destroy()
    A.destroy()


@pytest.mark.parametrize("lgs", [3, 5])
def test_device_setup_two_table_sizes(gpu, lgs):
    """The wave-shared ext+i fill and the RAP fill run the rows that fit a
    small table in one launch and the rest with the full table in another;
    with the small table at 2^3 / 2^5 slots (knob 19) both launches get rows
    on every Galerkin level, and every level still equals the host setup."""
    hv = gpu
    A = hv.ParCSRMatrix.laplacian27(20, 18, 16)
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=18)
    host = hv.BoomerAMG(**kw)
    host.setup_host(A)
    hv.set_knob(19, lgs)
    try:
        dev = hv.BoomerAMG(**kw)
        dev.setup(A)
    finally:
        hv.set_knob(19, 0)
    _same(_hier(hv, dev), _hier(hv, host))
    for s in (dev, host):
        s.destroy()
    A.destroy()


@pytest.mark.parametrize("lgcap", [5, 6])
def test_device_setup_host_rows(gpu, lgcap):
    """Tables capped at 32 / 64 slots (knob 7): the interpolation and Galerkin
    rows that outgrow them are finished by the host's row functions, and the
    result is still the host hierarchy byte for byte (the log counts them)."""
    hv = gpu
    A = hv.ParCSRMatrix.laplacian27(20, 18, 16)
    kw = hv.ij_amg_defaults(0)
    kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=18)
    hv.set_knob(7, lgcap)
    try:
        dev = hv.BoomerAMG(**kw)
        dev.setup(A)
    finally:
        hv.set_knob(7, 0)
    log = dev.setup_log()
    assert "rows on the host" in log, log
    host = hv.BoomerAMG(**kw)
    host.setup_host(A)
    _same(_hier(hv, dev), _hier(hv, host))
    dev.destroy()
    host.destroy()
    A.destroy()
