"""Join the counter passes of scripts/gpu_opprof.sh: per (kernel, grid) the mean
of every counter per dispatch, the mean duration, and derived columns.
  python scripts/pmc_ops_table.py <dir with pmc_*/ and trace/>

Derived (per dispatch):
  traffic_GB  2 * FETCH_SIZE + WRITE_SIZE (the gfx950 x2 read correction,
              MI355X_MICROARCH.md HBM section), GB
  L2hit%      TCC_HIT / (TCC_HIT + TCC_MISS)
  dram%       TCC_EA0_RDREQ_DRAM / TCC_EA0_RDREQ (read requests the L2 sends
              toward DRAM, Infinity Cache hits included, over all it sends)
  L2lat       TCP_TCC_READ_REQ_LATENCY / TCP_TCC_READ_REQ (cycles an L1 miss waits)
  TAbusy%     TA_TA_BUSY / (GRBM_GUI_ACTIVE x 32 CUs per XCD) (address unit busy)
  wait%       SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on waitcnt / barrier)
  vmem/wave   SQ_INSTS_VMEM_RD / SQ_WAVES
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

root = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)


def kname(s):
    s = s.replace("(anonymous namespace)::", "")
    s = re.sub(r"\(.*", "", s).replace("void hve::", "").replace("hve::", "")
    return s[:44]


for f in glob.glob(os.path.join(root, "pmc_*", "**", "run_counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        vals[(kname(r["Kernel_Name"]), int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in glob.glob(os.path.join(root, "trace", "**", "run_kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        dur[(kname(r["Kernel_Name"]), int(r.get("Grid_Size") or r["Grid_Size_X"]))].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)


def m(v, c):
    x = v.get(c)
    return sum(x) / len(x) if x else float("nan")


def q(a, b):
    return a / b if b else float("nan")


cols = ["us", "traffic_GB", "L2hit%", "dram%", "L2lat", "TAbusy%", "wait%", "vmem/wave", "lds/wave"]
print(f"{'kernel':44s} {'grid':>10s} " + " ".join(f"{c:>10s}" for c in cols))
keys = [k for k in vals if k[1] >= 100000]
for k in sorted(keys, key=lambda k: -m(vals[k], "FETCH_SIZE") if vals[k].get("FETCH_SIZE") else 0):
    v = vals[k]
    d = sum(dur[k]) / len(dur[k]) if dur.get(k) else float("nan")
    row = [d, (2 * m(v, "FETCH_SIZE") + m(v, "WRITE_SIZE")) * 1024 / 1e9,
           100 * q(m(v, "TCC_HIT_sum"), m(v, "TCC_HIT_sum") + m(v, "TCC_MISS_sum")),
           100 * q(m(v, "TCC_EA0_RDREQ_DRAM_sum"), m(v, "TCC_EA0_RDREQ_sum")),
           q(m(v, "TCP_TCC_READ_REQ_LATENCY_sum"), m(v, "TCP_TCC_READ_REQ_sum")),
           100 * q(m(v, "TA_TA_BUSY_sum"), m(v, "GRBM_GUI_ACTIVE") * 32),
           100 * q(m(v, "SQ_WAIT_ANY"), m(v, "SQ_WAVE_CYCLES")),
           q(m(v, "SQ_INSTS_VMEM_RD"), m(v, "SQ_WAVES")), q(m(v, "SQ_INSTS_LDS"), m(v, "SQ_WAVES"))]
    print(f"{k[0]:44s} {k[1]:10d} " + " ".join(f"{x:10.3f}" for x in row))
print("\nraw means per dispatch:")
for k in sorted(keys):
    print(k, {c: round(m(vals[k], c), 1) for c in sorted(vals[k])})
