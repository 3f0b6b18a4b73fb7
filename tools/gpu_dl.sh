#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python tools/dl_bench.py "$@" > gpurun_out/dl.json 2> gpurun_out/dl.err
rc=$?; echo "dl rc=$rc"; cat gpurun_out/dl.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/dl.err; exit $rc; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_dl -o run -- python $GRAFT_REPO_ROOT/tools/dl_bench.py "$@" > $GRAFT_REPO_ROOT/gpurun_out/prof_dl.log 2>&1
rc=$?; echo "prof rc=$rc"
rm -f $GRAFT_REPO_ROOT/gpurun_out/prof_dl/run_kernel_trace.csv
exit $rc
