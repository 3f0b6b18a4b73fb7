#!/bin/bash
# RANSAC PMC passes (one rocprofv3 run per counter group) over one C2 bench step; summary of the ransac kernels.
#   tools/gpu_pmc_ransac.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r03}
R=$GRAFT_REPO_ROOT
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmcr_${TAG}_$i -o run -- python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmcr_${TAG}_$i.log 2>&1)
  rc=$?; echo "pmc group $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/pmcr_${TAG}_$i.log; exit $rc; }
done
python $R/tools/pmc_summary.py $R/gpurun_out/pmcr_${TAG}_1 $R/gpurun_out/pmcr_${TAG}_2 > $R/gpurun_out/pmc_ransac_${TAG}.txt
rm -rf $R/gpurun_out/pmcr_${TAG}_1 $R/gpurun_out/pmcr_${TAG}_2  # raw CSVs exceed the copy-back cap
grep -i "ransac" $R/gpurun_out/pmc_ransac_${TAG}.txt
exit 0
