#!/bin/bash
# One PMC pass of LDS / VALU issue counters over the matchbench (distance GEMM). Usage: gpu_pmc_lds2.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-l}
R=$GRAFT_REPO_ROOT
for grp in "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INST_CYCLES_VMEM" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_EXP SQ_ACTIVE_INST_FLAT SQ_INSTS_SMEM SQ_LDS_ADDR_CONFLICT"; do
  name=$(echo $grp | cut -d' ' -f1)
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc_${TAG}_$name -o run -- python $R/tools/matchbench.py 100 > $R/gpurun_out/pmc_${TAG}_$name.log 2>&1)
  rc=$?; echo "pmc $name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/pmc_${TAG}_$name.log; continue; }
  python $R/tools/pmc_summary.py $R/gpurun_out/pmc_${TAG}_$name | grep mnn_pp
done
