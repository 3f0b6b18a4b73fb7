#!/bin/bash
# Two-variant A/B of the matcher kernel: matcher parity tests + bench for the in-tree library (A) and for
# gtsfm_amd/_lib/libgtsfm_hip_b.so (B, selected through GTSFM_HIP_LIB).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in A B; do
    if [ $v = B ]; then export GTSFM_HIP_LIB="$GRAFT_REPO_ROOT/gtsfm_amd/_lib/libgtsfm_hip_b.so"; fi
    timeout -k 10 300 python -u -m pytest tests/test_matcher_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_ab_$v.log 2>&1
    rc=$?; echo "$v: $(tail -1 gpurun_out/pytest_ab_$v.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_ab_$v.log; exit $rc; }
    timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_ab_$v.json 2> gpurun_out/bench_ab_$v.err
    rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_ab_$v.err; exit $rc; }
    python -c "import json; d=json.load(open('gpurun_out/bench_ab_$v.json')); print('$v', 'value', d['value'], 'stage', d['stage_ms'], 'kernel_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])"
done
