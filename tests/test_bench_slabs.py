"""bench.py's slab digests (CPU): the N = 1 line cuts its oracle-equal
iterate where an N-rank run's z-slabs end, and an N-rank line compares each
rank's sha256 with that cut.  The cut must be GenerateLaplacian's own
partition (hypre_GeneratePartitioning over z, par_laplace.c / par_laplace_27pt.c),
checked here against the library's partitioned generator on a loopback
communicator (no GPU needed to build the rank blocks)."""
import numpy as np
import pytest

import bench


@pytest.mark.parametrize("world", [2, 3, 4, 8])
@pytest.mark.parametrize("nx,ny,nz", [(8, 6, 16), (8, 6, 17), (5, 7, 23), (4, 4, 8), (16, 3, 9)])
@pytest.mark.parametrize("stencil", [7, 27])
def test_slab_cut_matches_generate_laplacian(hv, world, nx, ny, nz, stencil):
    if world > nz:
        pytest.skip("fewer planes than ranks")
    comms = hv.Comm.loopback(world)
    try:
        got = []
        for r in range(world):
            part = dict(comm=comms[r], P=1, Q=1, R=world, p=0, q=0, r=r)
            A = (hv.ParCSRMatrix.laplacian27(nx, ny, nz, **part) if stencil == 27
                 else hv.ParCSRMatrix.laplacian(nx, ny, nz, **part))
            got.append((A.first, A.n))
            A.destroy()
    finally:
        for c in comms:
            c.destroy()
    assert got == bench.slab_rows(nx, ny, nz, world)


def test_slab_digests_cut_the_whole_iterate():
    """Every N-column covers the iterate once, in rank order, and equal
    vectors give equal digests while one flipped bit changes exactly one."""
    nx, ny, nz = 8, 4, 19
    x = np.random.default_rng(3).standard_normal(nx * ny * nz)
    d = bench.slab_digests_of(x, nx, ny, nz)
    assert set(d) == {"1", "2", "4", "8"}
    for w in (2, 4, 8):
        cuts = bench.slab_rows(nx, ny, nz, w)
        assert cuts[0][0] == 0 and sum(c for _, c in cuts) == x.size
        assert all(f + c == g for (f, c), (g, _) in zip(cuts, cuts[1:]))
        assert d[str(w)] == [bench.sha256_f64(x[f:f + c]) for f, c in cuts]
    y = x.copy()
    y[nx * ny * 7] = np.nextafter(y[nx * ny * 7], np.inf)
    e = bench.slab_digests_of(y, nx, ny, nz)
    assert e["1"] != d["1"]
    assert sum(a != b for a, b in zip(e["8"], d["8"])) == 1
    # -0.0 and +0.0 are different bytes: the digest is of the bits
    z = np.zeros(4)
    assert bench.sha256_f64(z) != bench.sha256_f64(-z)


def test_digest_key_names_the_workload():
    import argparse
    a = argparse.Namespace(stencil=7, coef="1,1,1", agg=0, relax=18, coarsen=8, solver="amg")
    k = bench.digest_key(a, 512, 512, 512, 8)
    assert k == "512x512x512 stencil7 coef1,1,1 agg0 relax18 coarsen8 solveramg iters8"


def test_committed_digests_are_complete():
    """tests/golden/slab_digests.json (scripts/golden_digests.py from N = 1
    bench lines whose iterate equalled the oracle's): every workload carries
    the whole-iterate digest and the 2-, 4- and 8-slab columns."""
    import json
    import os
    with open(bench.GOLDEN_DIGESTS) as f:
        gold = json.load(f)
    assert "512x512x512 stencil7 coef1,1,1 agg0 relax18 coarsen8 solveramg iters8" in gold
    for key, d in gold.items():
        nz = int(key.split()[0].split("x")[2])
        for w in ("1", "2", "4", "8"):
            if int(w) <= nz:
                assert len(d[w]) == int(w) and all(len(h) == 64 for h in d[w]), (key, w)
    assert os.path.basename(bench.GOLDEN_DIGESTS) == "slab_digests.json"
