#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/matchbench.py 100 > gpurun_out/matchbench.log 2>&1 || exit $?
cat gpurun_out/matchbench.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run -- python $GRAFT_REPO_ROOT/tools/matchbench.py 100 > $GRAFT_REPO_ROOT/gpurun_out/prof1.log 2>&1 || exit $?
find $GRAFT_REPO_ROOT/gpurun_out/prof1 -name "*stats*" | head
