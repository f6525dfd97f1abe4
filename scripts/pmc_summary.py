"""Join rocprofv3 --pmc passes (FETCH_SIZE / WRITE_SIZE / TCC_HIT_sum,
TCC_MISS_sum) per (kernel, grid): mean counter per dispatch and mean duration.
FETCH_SIZE and WRITE_SIZE are reported in KiB.  Usage:
  python scripts/pmc_summary.py <dir_with_pmc_*> [min_grid]"""
import csv, glob, os, re, sys
from collections import defaultdict

root = sys.argv[1]
min_grid = int(sys.argv[2]) if len(sys.argv) > 2 else 0
vals = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for f in glob.glob(os.path.join(root, "pmc_*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void hve::", "").replace("hve::", "")
        key = (name[:40], int(r["Grid_Size"]))
        vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if r["Counter_Name"] in ("FETCH_SIZE",):
            dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
cols = ["FETCH_SIZE", "WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum"]
print(f"{'kernel':40s} {'grid':>10s} {'n':>3s} {'fetchMB':>9s} {'writeMB':>9s} {'L2hit%':>7s} {'us':>8s}")
for key in sorted(vals, key=lambda k: -max(vals[k].get("FETCH_SIZE", [0]))):
    if key[1] < min_grid:
        continue
    v = vals[key]
    m = lambda c: sum(v[c]) / len(v[c]) if v.get(c) else float("nan")
    hit = m("TCC_HIT_sum") / (m("TCC_HIT_sum") + m("TCC_MISS_sum")) * 100 if v.get("TCC_HIT_sum") else float("nan")
    d = sum(dur[key]) / len(dur[key]) if dur.get(key) else float("nan")
    print(f"{key[0]:40s} {key[1]:10d} {len(v.get('FETCH_SIZE', [])):3d} {m('FETCH_SIZE')*1024/1e6:9.1f} "
          f"{m('WRITE_SIZE')*1024/1e6:9.1f} {hit:7.1f} {d:8.1f}")
