#!/bin/bash
# PMC passes over one short bench step (separate rocprofv3 run per counter group), plus the counter list.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
(cd /tmp && timeout -k 10 60 rocprofv3 -L > $R/gpurun_out/counters_list.txt 2>&1) || echo "list rc=$?"
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES"; do
  name=$(echo $grp | cut -d' ' -f1)
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc_${TAG}_$name -o run -- python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc_${TAG}_$name.log 2>&1)
  rc=$?; echo "pmc $name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/pmc_${TAG}_$name.log; exit $rc; }
  python $R/tools/pmc_summary.py $R/gpurun_out/pmc_${TAG}_$name > $R/gpurun_out/pmc_${TAG}_$name.txt && rm -rf $R/gpurun_out/pmc_${TAG}_$name
done
