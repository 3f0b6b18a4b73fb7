"""Summarise rocprofv3 --pmc counter_collection CSVs: per kernel, dispatches and mean counter value per dispatch.

    python tools_pmc_summary.py <dir-with-run_counter_collection.csv> [...] > summary.txt
"""
import collections
import csv
import glob
import os
import sys


def main():
    rows = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                if "at::" in k or "rocclr" in k or "Cijk" in k:
                    continue
                rows[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    for k in sorted(rows, key=lambda k: -sum(rows[k].values())):
        n = max(len(disp[k]), 1)
        vals = " ".join(f"{c}={v / n:.4g}" for c, v in sorted(rows[k].items()))
        print(f"{k[:90]:90s} n={n:4d} {vals}")


if __name__ == "__main__":
    main()
