#!/bin/bash
# One GPU call: the GPU test suite, one bench line, and the rocprofv3 kernel stats of the same bench command.
#   tools/gpu_check.sh TAG [bench args...]      (run through gpurun; writes gpurun_out/*_TAG*)
# Every GPU step has its own time limit and the call stops at the first failing step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r02}
shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu --maxfail=5 -v --timeout 240 --timeout-method thread \
    > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_${TAG}.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/pytest_${TAG}.log | head -20; exit $rc; }
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke_${TAG}.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_${TAG}.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py "$@" > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_${TAG}.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_${TAG}.err; exit $rc; }
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}" \
    -o run -- python "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline "$@" \
    > "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}.log" 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd "$GRAFT_REPO_ROOT" && python tools/kstats.py "$(find gpurun_out/prof_${TAG} -name "*kernel_stats.csv" | sort | tail -n 1)"
exit 0
