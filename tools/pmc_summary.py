"""Summarise rocprofv3 --pmc counter_collection CSVs: per kernel, dispatches and mean counter value per dispatch.

    python tools/pmc_summary.py <dir-with-run_counter_collection.csv> [...] > summary.txt
    python tools/pmc_summary.py --json OUT.json --kernel mnn_pp_kernel <dirs...>
        -> {"hbm_bytes_per_launch": 2*FETCH_SIZE*1024 + WRITE_SIZE*1024, ...} for bench.py's roofline "traffic"
           (FETCH_SIZE doubled: gfx950 tallies 128-B reads at 64 B, MI355X_MICROARCH.md "HBM"; both in KiB)
    python tools/pmc_summary.py --json OUT.json --kernels a,b,c --steps N <dirs...>
        -> per kernel (substring match) the same per-launch bytes and dispatch count, plus the bytes of all of them
           per profiled step ("hbm_bytes_per_step", N = the bench steps the profiled command ran)
"""
import json
import collections
import csv
import glob
import os
import sys


def main():
    args = sys.argv[1:]
    out_json = kernel_sub = None
    if args[:1] == ["--json"]:
        out_json, args = args[1], args[2:]
    kernels_multi, n_steps = None, 1
    if args[:1] == ["--kernel"]:
        kernel_sub, args = args[1], args[2:]
    if args[:1] == ["--kernels"]:
        kernels_multi, args = args[1].split(","), args[2:]
    if args[:1] == ["--steps"]:
        n_steps, args = int(args[1]), args[2:]
    sys.argv = [sys.argv[0]] + args
    rows = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    cdisp = collections.defaultdict(set)  # per (kernel, counter): dispatches, for counters from separate passes
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                if "at::" in k or "rocclr" in k or "Cijk" in k:
                    continue
                rows[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
                cdisp[(k, r["Counter_Name"])].add((f, r.get("Dispatch_Id") or r.get("Correlation_Id")))
    def kernel_bytes(sub):
        ks = [k for k in rows if sub in k]
        tot = collections.defaultdict(float)
        cnt = collections.defaultdict(int)
        for k in ks:
            for c, v in rows[k].items():
                tot[c] += v
                cnt[c] += len(cdisp[(k, c)])
        per = {c: v / max(cnt[c], 1) for c, v in tot.items()}
        launches = max(cnt.values()) if cnt else 0
        return {"dispatches": dict(cnt), "counters_per_launch": per,
                "hbm_bytes_per_launch": 2 * per.get("FETCH_SIZE", 0.0) * 1024 + per.get("WRITE_SIZE", 0.0) * 1024,
                "hbm_bytes_total": 2 * tot.get("FETCH_SIZE", 0.0) * 1024 + tot.get("WRITE_SIZE", 0.0) * 1024,
                "launches": launches}

    if out_json and kernels_multi:
        res = {"kernels": {}, "steps_profiled": n_steps}
        for sub in kernels_multi:
            kb = kernel_bytes(sub)
            assert kb["launches"], f"no kernel matching {sub}"
            res["kernels"][sub] = kb
        res["hbm_bytes_per_step"] = sum(v["hbm_bytes_total"] for v in res["kernels"].values()) / n_steps
        json.dump(res, open(out_json, "w"), indent=1)
        print(json.dumps({k: (v["hbm_bytes_per_launch"], v["launches"]) for k, v in res["kernels"].items()}))
        return
    if out_json:
        ks = [k for k in rows if kernel_sub in k]
        assert ks, f"no kernel matching {kernel_sub}"
        tot = collections.defaultdict(float)
        cnt = collections.defaultdict(int)
        for k in ks:
            for c, v in rows[k].items():
                tot[c] += v
                cnt[c] += len(cdisp[(k, c)])
        per = {c: v / max(cnt[c], 1) for c, v in tot.items()}
        res = {"kernel": kernel_sub, "dispatches": dict(cnt), "counters_per_launch": per,
               "hbm_bytes_per_launch": 2 * per.get("FETCH_SIZE", 0.0) * 1024 + per.get("WRITE_SIZE", 0.0) * 1024}
        json.dump(res, open(out_json, "w"), indent=1)
        print(json.dumps(res))
        return
    for k in sorted(rows, key=lambda k: -sum(rows[k].values())):
        n = max(len(disp[k]), 1)
        vals = " ".join(f"{c}={v / n:.4g}" for c, v in sorted(rows[k].items()))
        print(f"{k[:90]:90s} n={n:4d} {vals}")


if __name__ == "__main__":
    main()
