"""Write tests/golden/ij_elast_A.npz from the reference's own test matrix
(src/test/TEST_ij/A.00000, A.00001: the 2-rank elasticity matrix that
TEST_ij/elast.jobs reads with `ij -fromfile A`).  Run here (the reference is
not on the GPU box); the tests read only the .npz.

Each row is assembled as HYPRE_IJMatrixRead + the aux-matrix assembly builds
it (IJ_mv/HYPRE_IJMatrix.c:1178 SetValues line by line; IJMatrix_parcsr.c:3032
puts the diagonal first, the other entries in file order), stacked rank by
rank; tests/ij_emul.py's rank emulation then splits each row into its own
and other-rank parts in that order."""
import os
import sys

import numpy as np

REF = "/root/reference/src/test/TEST_ij"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "ij_elast_A.npz")


def read_ij(prefix, nranks):
    indptr, indices, data, starts = [0], [], [], [0]
    for r in range(nranks):
        with open(f"{prefix}.{r:05d}") as fh:
            il, iu, _, _ = map(int, fh.readline().split())
            rows = {}
            for ln in fh:
                if ln.strip():
                    a, b, c = ln.split()
                    rows.setdefault(int(a), []).append((int(b), float(c)))
        for i in range(il, iu + 1):
            ent = rows.get(i, [])
            for j, v in [e for e in ent if e[0] == i] + [e for e in ent if e[0] != i]:
                indices.append(j)
                data.append(v)
            indptr.append(len(indices))
        starts.append(iu + 1)
    return (np.array(indptr, dtype=np.int32), np.array(indices, dtype=np.int32), np.array(data),
            np.array(starts, dtype=np.int32))


if __name__ == "__main__":
    if not os.path.isdir(REF):
        sys.exit("the reference tree is not here")
    ip, jj, vv, st = read_ij(os.path.join(REF, "A"), 2)
    np.savez_compressed(OUT, indptr=ip, indices=jj, data=vv, starts=st)
    print(OUT, len(ip) - 1, "rows", len(jj), "entries, starts", list(st))
