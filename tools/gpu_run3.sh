#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --images 24 --no-cpu-baseline > gpurun_out/bench_small.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -20 gpurun_out/bench_small.log
exit $rc
