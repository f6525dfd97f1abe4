"""The process-per-rank path across real process boundaries.

tests/mp_worker.py runs as world_size 2 and 3 under torch.distributed.run
(gloo bootstrap, 127.0.0.1 rendezvous).  Every rank is its own process with
its own HIP context, streams and library state; the communicator is the
host-staged shared-memory transport, because the box has one GPU and RCCL
refuses two ranks on one device.  The N-process iterates must equal a
one-GPU run under the rank emulation of the same N-rank setup bit for bit for
the 7- and 27-point operators, with coarse-level agglomeration off and on,
and for hybrid Gauss-Seidel across ranks.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_multiprocess_partitioned_solve_bitwise(world):
    env = dict(os.environ, OMP_NUM_THREADS="4", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(HERE, "mp_worker.py")]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and lines, f"rc={p.returncode}\nstdout:\n{p.stdout[-3000:]}\nstderr:\n{p.stderr[-3000:]}"
    res = json.loads(lines[-1])
    print(json.dumps(res, indent=1))
    assert res["ok"] and res["world"] == world
    assert all(c["bitwise"] for c in res["cases"])
