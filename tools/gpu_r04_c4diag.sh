#!/bin/bash
# C4 device-resident step time at 5 queued steps (persistent matcher outputs) + the all-pairs GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/c4diag; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_all_pairs_gpu.py tests/test_frontend_batched_gpu.py tests/test_c4_gpu.py > gpurun_out/c4diag/t.log 2>&1; rc=$?; tail -3 gpurun_out/c4diag/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/c4diag/s5.json 2> gpurun_out/c4diag/s5.err || exit $?
cut -c1-300 gpurun_out/c4diag/s5.json
