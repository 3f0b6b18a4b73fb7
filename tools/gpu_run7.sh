#!/bin/bash
# usage: gpu_run7.sh <pytest-target> <prof-name>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest ${1:-tests} -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_full.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_full.log | cut -c1-200; grep -o '"stage_ms[^}]*}' gpurun_out/bench_full.log
[ $rc -eq 0 ] || exit $rc
[ -n "$2" ] || exit 0
bash tools/gpu_prof.sh $2
