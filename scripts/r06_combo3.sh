# R_0 occupancy sweep, then the hybrid-GS cycle trace at 256^3
bash scripts/r06_r0pf.sh && bash scripts/r06_gstrace.sh
