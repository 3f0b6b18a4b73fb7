#!/bin/bash
# Matcher parity tests + the distance-GEMM microbench on one GPU (gpurun). Usage: gpu_match.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-m}
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_matcher_gpu.py \
    tests/test_lund_door_c1_gpu.py::test_lund_door_c1_all_pairs_vs_oracle_and_gt > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_${TAG}.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/matchbench.py 100 > gpurun_out/matchbench_${TAG}.json 2>&1
rc=$?; cat gpurun_out/matchbench_${TAG}.json; exit $rc
