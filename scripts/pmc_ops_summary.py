"""Mean of every collected counter per (kernel, grid) over the rocprofv3
--pmc passes of scripts/pmc_ops.sh, with the mean dispatch duration.

    python scripts/pmc_ops_summary.py [gpurun_out/pmcops]
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcops"
vals = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
    seen = set()
    for r in csv.DictReader(open(f)):
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("hve::", "")
        key = (name, int(r["Grid_Size"]))
        vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        did = (r.get("Dispatch_Id"), key)
        if did not in seen:
            seen.add(did)
            dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for key in sorted(vals, key=lambda k: -(sum(dur[k]) / max(1, len(dur[k])))):
    if not key[0].startswith("k_sell"):
        continue
    d = sum(dur[key]) / len(dur[key])
    print(f"{key[0]}  grid={key[1]}  {d:.1f} us (n={len(dur[key])})")
    for c, v in sorted(vals[key].items()):
        m = sum(v) / len(v)
        extra = f"  ({m * 1024 / 1e6:.1f} MB)" if c in ("FETCH_SIZE", "WRITE_SIZE") else ""
        print(f"    {c:32s} {m:16.1f}{extra}")
