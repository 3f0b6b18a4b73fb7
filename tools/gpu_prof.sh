#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=${1:-prof}
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/$OUT.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -2 $GRAFT_REPO_ROOT/gpurun_out/$OUT.log | cut -c1-300
exit $rc
