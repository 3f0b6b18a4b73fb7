#!/bin/bash
# PMC passes over a one-step bench run for the SIFT kernels (blur / extrema): VALU, LDS and wait breakdown, HBM bytes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-sift}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_SALU" "FETCH_SIZE" "WRITE_SIZE"; do
  name=$(echo $grp | cut -d' ' -f1)
  (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc_${TAG}_$name -o run -- python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc_${TAG}_$name.log 2>&1)
  rc=$?; echo "pmc $name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/pmc_${TAG}_$name.log; exit $rc; }
  python $R/tools/pmc_summary.py $R/gpurun_out/pmc_${TAG}_$name > $R/gpurun_out/pmc_${TAG}_$name.txt
  rm -rf $R/gpurun_out/pmc_${TAG}_$name
done
