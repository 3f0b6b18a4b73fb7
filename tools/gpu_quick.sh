#!/bin/bash
# Quick GPU check: selected test files (args) + a short bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest "$@" -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_quick.log | tail -30
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" gpurun_out/pytest_quick.log | tail -60; exit $rc; }
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_quick.json; [ $rc -eq 0 ] || tail -20 gpurun_out/bench_quick.err
exit $rc
