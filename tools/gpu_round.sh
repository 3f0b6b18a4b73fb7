#!/bin/bash
# Short bench line (kernel-timed roofline) + rocprofv3 kernel stats + PMC passes, for one tag.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_${TAG}.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_${TAG}.err; exit $rc; }
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG} -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd "$GRAFT_REPO_ROOT" && bash tools/gpu_pmc_mnn.sh ${TAG}
