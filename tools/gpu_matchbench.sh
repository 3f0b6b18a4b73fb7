#!/bin/bash
# Distance-GEMM microbench + its rocprofv3 kernel stats (gpurun). Usage: gpu_matchbench.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-mb}
timeout -k 10 120 python -u tools/matchbench.py 100 > gpurun_out/matchbench_${TAG}.json 2>gpurun_out/matchbench_${TAG}.err
rc=$?; cat gpurun_out/matchbench_${TAG}.json; [ $rc -eq 0 ] || { tail gpurun_out/matchbench_${TAG}.err; exit $rc; }
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run -- python3 tools/matchbench.py 100 \
    > gpurun_out/prof_${TAG}.log 2>&1
rc=$?; f=$(find gpurun_out/prof_${TAG} -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -8 "$f"; exit $rc
