#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over a short run; writes the per-kernel summaries and
# gpurun_out/<TAG>_mnn_pmc.json (HBM bytes per distance-GEMM launch, read by bench.py's roofline "traffic").
# Usage: gpu_pmc_mnn.sh TAG [bench|matchbench] [config: c2 (default) | c1 | c4 ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r01}
WHAT=${2:-bench}
CFG=${3:-c2}
R=$GRAFT_REPO_ROOT
if [ "$WHAT" = "bench" ]; then CMD="$R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --config $CFG"; else CMD="$R/tools/matchbench.py 100"; fi
dirs=""
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES SQ_WAIT_ANY SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM"; do
  name=$(echo $grp | cut -d' ' -f1)
  (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc_${TAG}_$name -o run -- python $CMD > $R/gpurun_out/pmc_${TAG}_$name.log 2>&1)
  rc=$?; echo "pmc $name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/pmc_${TAG}_$name.log; exit $rc; }
  python $R/tools/pmc_summary.py $R/gpurun_out/pmc_${TAG}_$name > $R/gpurun_out/pmc_${TAG}_$name.txt
  dirs="$dirs $R/gpurun_out/pmc_${TAG}_$name"
done
python $R/tools/pmc_summary.py --json $R/gpurun_out/${TAG}_${CFG}_mnn_pmc.json --kernel mnn_pp_kernel $dirs && rm -rf $dirs
cat $R/gpurun_out/pmc_${TAG}_*.txt | grep -A3 mnn_pp | head -40
