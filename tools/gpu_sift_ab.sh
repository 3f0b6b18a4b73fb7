#!/bin/bash
# SIFT parity tests + a short bench line + kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_sift_gpu.py tests/test_frontend_batched_gpu.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_sab.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_sab.log | tail -12; [ $rc -eq 0 ] || { grep -B5 -A25 "Error\|assert" gpurun_out/pytest_sab.log | tail -50; exit $rc; }
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_sab.json 2> gpurun_out/bench_sab.err
rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_sab.err; exit $rc; }
python -c "import json; d=json.load(open('gpurun_out/bench_sab.json')); print('value', d['value'], 'ms', d['ms_per_step'], 'stage', d['stage_ms'])"
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_sab -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_sab.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python $GRAFT_REPO_ROOT/tools/kstats.py $GRAFT_REPO_ROOT/gpurun_out/prof_sab/run_kernel_stats.csv > $GRAFT_REPO_ROOT/gpurun_out/kstats_sab.txt; head -16 $GRAFT_REPO_ROOT/gpurun_out/kstats_sab.txt
