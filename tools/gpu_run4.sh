#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_verifier_gpu.py -x -q -m gpu > gpurun_out/pytest_ver.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_ver.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_full.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_full.log
[ $rc -eq 0 ] || exit $rc
exit 0
rc=$?; echo "prof rc=$rc"
find $GRAFT_REPO_ROOT/gpurun_out/prof3 -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-160 | head -30
exit $rc
