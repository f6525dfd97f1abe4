# A/B of the dictionary-loop variants, then the one-GPU references of the
# default workload's 2 / 4 / 8-rank lines (see r06_ab_dictw.sh, r06_refs.sh).
bash scripts/r06_ab_dictw.sh 07_ab_dictw && REF_TIMEOUT=330 bash scripts/r06_refs.sh 05_refs7 "--n 512" 2 4 8
