"""Timeline of one SIFT extraction from a rocprofv3 kernel_trace.csv: every kernel from the chosen launch of the u8
base blur (the first SIFT kernel of an extraction) to the descriptor kernel, with start / end in microseconds
relative to the base blur's start and the queue it ran on, so the critical path through the octaves is visible.

    python tools/sift_timeline.py <kernel_trace.csv> [which: index of the base-blur launch, default -2]
"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
which = int(sys.argv[2]) if len(sys.argv) > 2 else -2
starts = [i for i, r in enumerate(rows) if "blur2d_kernel<5, true>" in r["Kernel_Name"]]
i0 = starts[which]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:]:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:44]
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    q = r.get("Queue_Id", r.get("Stream_Id", "?"))
    print(f"{s:9.1f} {e:9.1f} {e - s:8.1f}  q{q:>3}  {name}")
    if "descriptor_kernel" in name:
        break
