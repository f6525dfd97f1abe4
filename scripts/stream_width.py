"""Read/write-mix streams with 8-B and 16-B accesses per lane (hypreve_BenchStream
-R with knob 3 = 0 | 2): what the access width is worth at each mix."""
import ctypes as C
import json
import sys

sys.path.insert(0, "hypre-ve_amd")
import hypreve as hv

hv.init()
n = 1 << 27
for R in (1, 2, 5):
    row = {"reads": R}
    for width, kv in ((8, 0), (16, 2)):
        hv.set_knob(3, kv)
        ms = C.c_double()
        hv.check(hv.lib().hypreve_BenchStream(-R, C.c_int64(n), 20, C.byref(ms)), "BenchStream")
        row[f"{width}B_GBs"] = round((R + 1) * 8 * n / ms.value / 1e6, 1)
    print(json.dumps(row), flush=True)
hv.set_knob(3, 0)
