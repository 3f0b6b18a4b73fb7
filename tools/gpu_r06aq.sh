#!/bin/bash
# RANSAC occupancy evidence: PMC passes over one C2 step (tools/gpu_pmc_ransac.sh) and a kernel trace whose per-dispatch
# VGPR / AGPR / LDS / workgroup columns give each RANSAC kernel's register- and LDS-bound waves per SIMD.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/gpu_pmc_ransac.sh r06aq || exit $?
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r06aq_tr -o run -- python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/r06aq_tr.log 2>&1)
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
python tools/ransac_occupancy.py "$(find gpurun_out/r06aq_tr -name '*kernel_trace.csv' | head -1)" gpurun_out/pmc_ransac_r06aq.txt > gpurun_out/r06aq_ransac_occupancy.md
cat gpurun_out/r06aq_ransac_occupancy.md
rm -rf gpurun_out/r06aq_tr
