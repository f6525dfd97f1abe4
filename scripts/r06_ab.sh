# A/B of the lane-packed layouts at 512^3 on one MI355X: R_0's codes per lane
# load (HVE_CODE_PACK 1 / 4 / 8) and the dictionary streams (HVE_DICT_WIDE 0 / 1),
# one process per variant (the switches are read once), scripts/ops_time.py.
set -o pipefail
OUT=gpurun_out/r06/${1:-04_ab}
N=${2:-512}
mkdir -p $OUT
HVE_CODE_PACK=1 HVE_DICT_WIDE=0 timeout -k 10 200 python -u scripts/ops_time.py $N > $OUT/pack1_wide0.txt 2>&1 && \
HVE_CODE_PACK=4 timeout -k 10 200 python -u scripts/ops_time.py $N > $OUT/pack4_wide1.txt 2>&1 && \
HVE_CODE_PACK=8 timeout -k 10 200 python -u scripts/ops_time.py $N > $OUT/pack8_wide1.txt 2>&1
echo "exit $?"
