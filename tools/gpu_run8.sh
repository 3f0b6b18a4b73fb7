#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_verifier_gpu.py -x -q -m gpu > gpurun_out/pytest_ver.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ver.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ransac_phases.py > gpurun_out/phases.log 2>&1
rc=$?; echo "phases rc=$rc"; cat gpurun_out/phases.log | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_full.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -o '"value[^,]*,' gpurun_out/bench_full.log; grep -o '"stage_ms[^}]*}' gpurun_out/bench_full.log
exit $rc
