#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over a short bench run; writes the per-kernel summaries and
# gpurun_out/<TAG>_mnn_pmc.json (HBM bytes per distance-GEMM launch, read by bench.py's roofline "traffic").
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
dirs=""
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES SQ_WAIT_ANY SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE"; do
  name=$(echo $grp | cut -d' ' -f1)
  (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc_${TAG}_$name -o run -- python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc_${TAG}_$name.log 2>&1)
  rc=$?; echo "pmc $name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/pmc_${TAG}_$name.log; exit $rc; }
  python $R/tools/pmc_summary.py $R/gpurun_out/pmc_${TAG}_$name > $R/gpurun_out/pmc_${TAG}_$name.txt
  dirs="$dirs $R/gpurun_out/pmc_${TAG}_$name"
done
python $R/tools/pmc_summary.py --json $R/gpurun_out/${TAG}_mnn_pmc.json --kernel mnn_mfma_kernel $dirs && rm -rf $dirs
