"""One rank of tests/test_gpu_multiprocess.py, launched by
`python -m torch.distributed.run --nproc-per-node N ... tests/mp_worker.py`.

Each process is one rank of the process-per-GPU path: torch.distributed (gloo)
bootstraps, the ranks build their z-slab of the Laplacian through
GenerateLaplacian[27pt] with the communicator, set up (distributed setup:
every rank builds its own rows of each level) and solve.  The ranks share
the box's single GPU, which RCCL refuses, so the communicator is the
host-staged shared-memory transport (hypreve_CommCreateShm); every other line
of the data path -- operator split, halo exchange on the side stream,
agglomerated coarse levels, coarse solve, the distributed setup's all-to-alls
-- is the production code.  Rank 0 then solves the same problem on one GPU
without a communicator under the rank emulation of the same N-rank setup
(hypreve_BoomerAMGSetRankEmulation: hypre's N-process rules, the contract of
every N-rank run) and compares the gathered iterate bit for bit.
Prints one JSON line on rank 0; exits nonzero on any mismatch.
"""
import json
import os
import sys
import uuid

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hypre-ve_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (slab cut and digests of the bench's N-rank parity)


def gen(hv, stencil, nx, ny, nz, **part):
    if stencil == 27:
        return hv.ParCSRMatrix.laplacian27(nx, ny, nz, **part)
    return hv.ParCSRMatrix.laplacian(nx, ny, nz, **part)


def main():
    import torch
    import torch.distributed as dist

    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    import hypreve as hv

    torch.cuda.set_device(0)
    hv.init()
    names = [f"/hve_mp_{uuid.uuid4().hex[:12]}"] if rank == 0 else [None]
    dist.broadcast_object_list(names, 0)
    comm = hv.Comm.shm(rank, world, names[0])
    comm.self_test()

    cases = [
        # (stencil, nx, ny, nz, relax, agglo_rows, num_blocks)
        (7, 18, 16, 10 * world, 18, 0, 1),
        (7, 18, 16, 10 * world, 18, 2000, 1),
        (27, 14, 13, 8 * world, 18, 0, 1),
        (27, 14, 13, 8 * world, 18, 2000, 1),
        (7, 16, 15, 9 * world, 13, 0, 2),
    ]
    results, ok = [], True
    for stencil, nx, ny, nz, relax, agglo, nb in cases:
        kw = hv.ij_amg_defaults(0)
        kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=relax, tol=1e-8, max_iter=60,
                  agglo_rows=agglo, num_blocks=nb)
        N = nx * ny * nz
        rng = np.random.default_rng(1000 + stencil + agglo + relax)
        b_glob = rng.standard_normal(N)
        A = gen(hv, stencil, nx, ny, nz, comm=comm, P=1, Q=1, R=world, p=0, q=0, r=rank)
        amg = hv.BoomerAMG(**kw)
        amg.setup(A)
        b = hv.ParVector(A.n, b_glob[A.first:A.first + A.n], comm=comm, first=A.first, global_n=N)
        x = hv.ParVector(A.n, np.zeros(A.n), comm=comm, first=A.first, global_n=N)
        it, rr = amg.solve(A, b, x)
        xl = x.get()
        part = (A.first, xl, it, rr, amg.num_levels(), bench.sha256_f64(xl))
        gathered = [None] * world
        dist.all_gather_object(gathered, part)
        if rank == 0:
            gathered.sort(key=lambda o: o[0])
            starts = [o[0] for o in gathered] + [N]
            xN = np.concatenate([o[1] for o in gathered])
            A1 = gen(hv, stencil, nx, ny, nz)
            a1 = hv.BoomerAMG(**kw)
            a1.set_rank_emulation(starts)  # the N-rank setup (and hybrid-GS row blocks) on one GPU
            a1.setup(A1)
            b1 = hv.ParVector(N, b_glob)
            x1 = hv.ParVector(N, np.zeros(N))
            it1, rr1 = a1.solve(A1, b1, x1)
            x1h = x1.get()
            same = bool(np.array_equal(x1h, xN))
            # bench.py's N-rank parity: each rank's sha256 against the emulated
            # one-GPU iterate cut at GenerateLaplacian's slab boundaries
            cut = bench.slab_rows(nx, ny, nz, world)
            digests_ok = [o[0] for o in gathered] == [f for f, _ in cut] and \
                [o[5] for o in gathered] == [bench.sha256_f64(x1h[f:f + c]) for f, c in cut]
            same = same and digests_ok
            its = [o[2] for o in gathered]
            good = same and all(i == it1 for i in its) and all(abs(o[3] - rr1) <= 1e-10 * rr1 for o in gathered) \
                and gathered[0][4] == a1.num_levels()
            ok = ok and good
            results.append({"stencil": stencil, "grid": [nx, ny, nz], "relax": relax, "agglo_rows": agglo,
                            "num_blocks": nb, "iters": its, "iters_1rank": it1, "rel_res": rr1,
                            "levels": a1.num_levels(), "bitwise": same, "slab_digests": digests_ok, "ok": good})
            for o in (a1, A1, b1, x1):
                o.destroy()
        for o in (amg, A, b, x):
            o.destroy()
        flag = [ok]
        dist.broadcast_object_list(flag, 0)
        ok = flag[0]
    if rank == 0:
        print(json.dumps({"world": world, "transport": "shm", "ok": ok, "cases": results}), flush=True)
    comm.destroy()
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
