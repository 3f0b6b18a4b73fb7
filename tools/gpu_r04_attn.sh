#!/bin/bash
# SuperGlue attention change: the SuperGlue / deep-engine GPU tests, then the C5 slice bench and its kernel grid.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-attn}
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_superglue_gpu.py tests/test_deep_frontend_gpu.py > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_${TAG}.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_${TAG}.log | head -20; exit $rc; }
timeout -k 10 400 python -u bench.py --config c5 --no-cpu-baseline > gpurun_out/bench_${TAG}_c5.json 2> gpurun_out/bench_${TAG}_c5.err
rc=$?; cut -c1-400 gpurun_out/bench_${TAG}_c5.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_${TAG}_c5.err; exit $rc; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['stage_ms'], d['roofline']['frac'])" gpurun_out/bench_${TAG}_c5.json
