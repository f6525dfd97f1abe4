import sys; sys.path.insert(0,'hypre-ve_amd')
import hypreve as hv
hv.init()
A = hv.ParCSRMatrix.laplacian27(64,66,64)
kw = hv.ij_amg_defaults(0); kw.update(coarsen_type=8, relax_type=18, P_max_elmts=4)
amg = hv.BoomerAMG(**kw); amg.setup(A)
print("layout", amg.level_layout(0,0), amg.level_layout(0,2), amg.fused_resid_restrict(), flush=True)
