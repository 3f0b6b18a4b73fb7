"""Print the kernel timeline of the last bench step from a rocprofv3 kernel_trace.csv (from the last `anchor` kernel)."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
anchor = sys.argv[2] if len(sys.argv) > 2 else "ransac_init"
last = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]][-1]
t0 = int(rows[last]["Start_Timestamp"])
for r in rows[last - int(sys.argv[3] if len(sys.argv) > 3 else 0):last + 60]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("%-44s %9.1f %8.1f  grid %s x %s" % (r["Kernel_Name"][:44], (s - t0) / 1e3, (e - s) / 1e3, r["Grid_Size_X"],
                                              r["Grid_Size_Y"]))
