# R_0's jagged product-parallel loop (parity tests, A/B), then configs[4]'s
# and the 27-point operator's references (r06_ab_r0.sh, r06_refs2.sh).
bash scripts/r06_ab_r0.sh 09_r0pw | tail -1 | grep -q "exit 0" || { echo "exit 1 (r0pw)"; exit 1; }
bash scripts/r06_refs2.sh
