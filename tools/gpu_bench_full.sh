#!/bin/bash
# Round bench: default bench.py line (with cpu_baseline) + rocprofv3 kernel stats of the same command.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r01}
timeout -k 10 900 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_${TAG}.json
[ $rc -eq 0 ] || { tail -20 gpurun_out/bench_${TAG}.err; exit $rc; }
cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG} -o run -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}.log | cut -c1-300
exit $rc
