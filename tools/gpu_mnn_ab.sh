#!/bin/bash
# A/B timing of the matcher kernel: matcher parity tests + 3 bench runs (kernel-only roofline line).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_matcher_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_ab.log; exit $rc; }
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err
rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_ab.err; exit $rc; }
python -c "import json; d=json.load(open('gpurun_out/bench_ab.json')); print('value', d['value'], 'stage', d['stage_ms'], 'kernel_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])"
