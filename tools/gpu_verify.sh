#!/bin/bash
# Verifier GPU tests + one C2 bench line with kernel stats (gpurun). Usage: gpu_verify.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-v}
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_verifier_gpu.py \
    tests/test_sampson_known_answers.py tests/test_lund_door_c1_gpu.py > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_${TAG}.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/pytest_${TAG}.log | head; exit $rc; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}" \
    -o run -- python "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/bench_${TAG}.json" 2>&1
rc=$?; cd "$GRAFT_REPO_ROOT"; grep -o '"stage_ms": {[^}]*}' gpurun_out/bench_${TAG}.json; grep -o '"value": [0-9.]*' gpurun_out/bench_${TAG}.json | head -1
python tools/kstats.py "$(find gpurun_out/prof_${TAG} -name "*kernel_stats.csv" | sort | tail -n 1)" | grep ransac
exit $rc
