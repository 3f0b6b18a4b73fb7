"""Per-(kernel, grid) launch durations from a rocprofv3 kernel_trace.csv (development tool).
    python tools/kgrid.py run_kernel_trace.csv [name-substring ...]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
keys = sys.argv[2:] or [""]
agg = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    if not any(k in n for k in keys):
        continue
    g = (r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
    agg[(n[:48], g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (n, g), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"{n:48s} grid {'x'.join(g):22s} {len(v):5d} x {sum(v) / len(v):9.1f} us = {sum(v) / 1e3:9.2f} ms")
