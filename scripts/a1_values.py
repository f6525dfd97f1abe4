# Distinct values per group of 256 consecutive rows of the level-1 operator
# (host setup on the CPU): is a per-group value table worth it?
import sys, numpy as np
sys.path.insert(0, "hypre-ve_amd")
import hypreve as hv
n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
A = hv.ParCSRMatrix.laplacian(n, n, n)
kw = hv.ij_amg_defaults(0)
kw.update(coarsen_type=8, interp_type=6, P_max_elmts=4, relax_type=18)
amg = hv.BoomerAMG(**kw)
amg.setup_host(A)
for lev in (1, 2):
    ip, jj, vv, (nr, nc) = amg.level_matrix(lev, 0)
    bits = vv.view(np.int64)
    tot_d = 0; tot_e = 0; mx = 0
    for g0 in range(0, nr, 256):
        g1 = min(nr, g0 + 256)
        b = bits[ip[g0]:ip[g1]]
        d = len(np.unique(b)); tot_d += d; tot_e += len(b); mx = max(mx, d)
    print(f"level {lev}: rows {nr} nnz {len(vv)} distinct overall {len(np.unique(bits))} per-group mean {tot_d/((nr+255)//256):.0f} max {mx} entries/group {tot_e/((nr+255)//256):.0f}")
