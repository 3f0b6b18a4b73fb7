#!/bin/bash
# Round check on the GPU box: gpu parity tests, smoke, default bench line, rocprofv3 kernel stats of the bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_${TAG}.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_${TAG}.log
[ $rc -eq 0 ] || exit $rc
bash gpu_bench_full.sh ${TAG}
