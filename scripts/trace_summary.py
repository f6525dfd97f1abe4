"""Per (kernel, grid) summary of a rocprofv3 kernel trace: mean duration and
count, sorted by total time.  Usage: python scripts/trace_summary.py trace.csv [min_calls]"""
import csv, re, sys
from collections import defaultdict

path = sys.argv[1]
min_calls = int(sys.argv[2]) if len(sys.argv) > 2 else 10
acc = defaultdict(list)
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"]
    m = re.search(r"k_sell<(\d+), (\w+)>|k_sellILi(\d)ELb(\d)", name)
    short = re.sub(r"\(.*", "", name)
    short = re.sub(r"void hve::", "", short)
    key = (short[:60], int(r["Grid_Size_X"]))
    acc[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
rows = [(k, len(v), sum(v) / len(v), sum(v)) for k, v in acc.items() if len(v) >= min_calls]
rows.sort(key=lambda x: -x[3])
tot = sum(x[3] for x in rows)
print(f"{'kernel':60s} {'grid':>10s} {'n':>5s} {'mean_us':>9s} {'tot_ms':>8s} {'%':>5s}")
for (name, grid), n, mean, s in rows:
    print(f"{name:60s} {grid:10d} {n:5d} {mean:9.1f} {s/1e3:8.2f} {100*s/tot:5.1f}")
