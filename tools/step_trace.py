"""Kernel time of the last front-end step in a rocprofv3 kernel_trace.csv: from the last launch of the anchor kernel
(default: the first SIFT kernel of an extraction, gray_pad_kernel or the u8 base blur) to the end of the trace, per kernel name (count,
busy ms) plus the idle gaps between consecutive kernels.

    python tools/step_trace.py <kernel_trace.csv> [anchor] [end_anchor]
"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
anchor = sys.argv[2] if len(sys.argv) > 2 else None
if anchor is None:  # the first SIFT kernel of an extraction: the gray staging (round 6), else the u8 base blur
    anchor = "gray_pad_kernel" if any("gray_pad_kernel" in r["Kernel_Name"] for r in rows) else "blur2d_kernel<5, true>"
starts = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
i0 = starts[-2] if len(starts) > 1 else starts[-1]  # the last full step (the final one may be instrumented)
i1 = starts[-1] if len(starts) > 1 else len(rows)
if len(sys.argv) > 3:
    i1 = next(i for i in range(i0 + 1, len(rows)) if sys.argv[3] in rows[i]["Kernel_Name"]) + 1
step = rows[i0:i1]
t0, t_end = int(step[0]["Start_Timestamp"]), max(int(r["End_Timestamp"]) for r in step)
busy = collections.defaultdict(lambda: [0, 0.0])
gap, last_end = 0.0, t0
for r in step:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    name = name.split("(")[0][:60]
    busy[name][0] += 1
    busy[name][1] += (e - s) / 1e6
    if s > last_end:
        gap += (s - last_end) / 1e6
    last_end = max(last_end, e)
print(f"step span {(t_end - t0) / 1e6:.3f} ms, {len(step)} kernels, idle gaps {gap:.3f} ms")
for name, (n, ms) in sorted(busy.items(), key=lambda kv: -kv[1][1]):
    print(f"  {name:60s} {n:5d} {ms:9.3f} ms")
