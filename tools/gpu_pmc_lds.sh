#!/bin/bash
# One extra PMC pass (LDS / VALU / wait counters) over a short bench run; per-kernel summary.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
grp="SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_VMEM"
(cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc_${TAG}_lds -o run -- python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc_${TAG}_lds.log 2>&1)
rc=$?; echo "pmc lds rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/pmc_${TAG}_lds.log; exit $rc; }
python $R/tools/pmc_summary.py $R/gpurun_out/pmc_${TAG}_lds > $R/gpurun_out/pmc_${TAG}_lds.txt && rm -rf $R/gpurun_out/pmc_${TAG}_lds
