#!/bin/bash
# Full round check on one MI355X: every GPU test, smoke(), the default bench line (with cpu_baseline), then the
# rocprofv3 kernel stats + HBM PMC passes for the profile tag (gpu_round.sh without its short bench).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 gpurun_out/pytest_${TAG}.log)"; [ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_${TAG}.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1
rc=$?; echo "smoke rc=$rc: $(tail -1 gpurun_out/smoke_${TAG}.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/smoke_${TAG}.log; exit $rc; }
timeout -k 10 400 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_${TAG}.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_${TAG}.err; exit $rc; }
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG} -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd "$GRAFT_REPO_ROOT" && bash tools/gpu_pmc_mnn.sh ${TAG}
