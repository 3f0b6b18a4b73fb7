"""Per-kernel achieved HBM-side bandwidth: (2 x FETCH_SIZE + WRITE_SIZE) per step from the tools/gpu_pmc_hbm.sh
summaries over kernel time per step from a rocprofv3 --stats CSV of the same bench command.
    python tools/hbm_table.py <FETCH.txt> <WRITE.txt> <kernel_stats.csv> <pmc step runs> <stats step runs>"""
import csv
import re
import sys


def pmc(path):
    out = {}
    for line in open(path):
        m = re.match(r"(.*?)\s+n=\s*(\d+)\s+\w+=([0-9.e+]+)", line)
        if m:
            out[m.group(1).strip()] = (int(m.group(2)), float(m.group(3)))
    return out


fetch, write = pmc(sys.argv[1]), pmc(sys.argv[2])
pmc_steps, stat_steps = int(sys.argv[4]), int(sys.argv[5])
rows = []
for r in csv.DictReader(open(sys.argv[3])):
    name = r["Name"]
    if "rocblas" in name or "at::" in name:  # scene rendering by torch, outside the timed step
        continue
    key = next((k for k in fetch if name.startswith(k) or k.startswith(name[:60])), None)
    if key is None or key not in write:
        continue
    n, f = fetch[key]
    _, w = write[key]
    bytes_step = (2 * f + w) * n * 1024 / pmc_steps  # KB per launch (FETCH doubled: gfx950 tallies 128-B reads at 64 B)
    ms_step = float(r["TotalDurationNs"]) / 1e6 / stat_steps
    rows.append((ms_step, name[:70], bytes_step / 1e9, bytes_step / (ms_step * 1e-3) / 1e12))
rows.sort(reverse=True)
print("| kernel | ms/step | HBM-side GB/step | TB/s | of 8 TB/s |")
print("|---|---|---|---|---|")
for ms, name, gb, tbs in rows[:16]:
    print(f"| `{name}` | {ms:.2f} | {gb:.2f} | {tbs:.2f} | {tbs / 8:.0%} |")
