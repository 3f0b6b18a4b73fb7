#!/bin/bash
# HBM bytes per kernel over a one-step bench run (FETCH_SIZE and WRITE_SIZE, one rocprofv3 pass each).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-hbm}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc_${TAG}_$grp -o run -- python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc_${TAG}_$grp.log 2>&1)
  rc=$?; echo "pmc $grp rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/pmc_${TAG}_$grp.log; exit $rc; }
  python $R/tools/pmc_summary.py $R/gpurun_out/pmc_${TAG}_$grp > $R/gpurun_out/pmc_${TAG}_$grp.txt
  rm -rf $R/gpurun_out/pmc_${TAG}_$grp
done
