"""Per RANSAC kernel: registers, LDS and the waves per SIMD they allow (MI355X: 512 VGPR+AGPR per lane per SIMD in
granules of 8, 160 KiB LDS per CU, 4 SIMDs per CU, at most 8 waves per SIMD), from a rocprofv3 kernel trace; plus the
PMC summary's per-dispatch counters (tools/gpu_pmc_ransac.sh) and the mean resident waves per SIMD they imply:
SQ_WAVE_CYCLES x 4 (the counter counts quad-cycles, MI355X_MICROARCH.md) / (mean launch us x clock x 1024 SIMDs).
The trace's register and LDS columns can omit AGPRs and dynamic LDS; the code object's notes are authoritative
(profiles/r06aq_ransac_occupancy/README.md takes them from there).

    python tools/ransac_occupancy.py <kernel_trace.csv> <pmc_ransac_summary.txt> > table.md
"""
import collections
import csv
import re
import sys

N_SIMD = 256 * 4
CLOCK_MHZ = 2000  # profiled runs hold ~1.9-2.0 GHz (MI355X_MICROARCH.md)


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    pmc = {}
    for line in open(sys.argv[2]):
        m = re.match(r"(.*?) n=\s*(\d+) (.*)", line.strip())
        if m and "ransac" in m.group(1):
            pmc[m.group(1)[:60]] = dict(kv.split("=") for kv in m.group(3).split())
    seen = collections.OrderedDict()
    dur = collections.defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"]
        if "ransac" not in name:
            continue
        short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        dur[short].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        if short not in seen:
            seen[short] = r
    print("| kernel | arch VGPR | AGPR | LDS B | WG threads | waves/SIMD (regs) | WGs/CU (LDS) | waves/SIMD (bound) |"
          " mean us | PMC mean resident waves/SIMD |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for short, r in seen.items():
        v, a = int(r["VGPR_Count"]), int(r["Accum_VGPR_Count"])
        lds = int(r["LDS_Block_Size"])
        wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
        alloc = -(-(v + a) // 8) * 8
        w_regs = min(8, 512 // max(alloc, 1))
        waves_per_wg = -(-wg // 64)
        wg_lds = 160 * 1024 // lds if lds else 10 ** 9
        w_lds = wg_lds * waves_per_wg / 4
        bound = min(w_regs, w_lds, 8)
        occ = "-"
        mean_us = sum(dur[short]) / len(dur[short])
        for k, d in pmc.items():
            if short.split("<")[0] in k and "SQ_WAVE_CYCLES" in d:
                occ = f"{float(d['SQ_WAVE_CYCLES']) * 4 / (mean_us * CLOCK_MHZ * N_SIMD):.2f}"
        print(f"| {short} | {v} | {a} | {lds} | {wg} | {w_regs} | {wg_lds if lds else '-'} | {bound:g} | "
              f"{sum(dur[short]) / len(dur[short]):.1f} | {occ} |")


if __name__ == "__main__":
    main()
