#!/bin/bash
# Split-precision deep nets check: the SuperPoint / SuperGlue / deep GPU tests, then the C5 and C3 benches under a
# kernel-stats trace.   tools/gpu_r04_sg.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r04sg}
timeout -k 10 500 python -u -m pytest tests/test_superpoint_gpu.py tests/test_superglue_gpu.py tests/test_deep_frontend_gpu.py -v --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/${TAG}_tests.log | tail -40; [ $rc -eq 0 ] || { grep -B5 -A30 "Error\b\|assert" gpurun_out/${TAG}_tests.log | head -120; exit $rc; }
for cfg in c5 c3; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_$cfg -o run -- python -u bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_$cfg.json 2> gpurun_out/${TAG}_$cfg.err
  rc=$?; cut -c1-600 gpurun_out/${TAG}_$cfg.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_$cfg.err; exit $rc; }
  f=$(find gpurun_out/${TAG}_$cfg -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/${TAG}_${cfg}_kernel_stats.csv; python tools/kstats.py $f | head -14; rm -rf gpurun_out/${TAG}_$cfg
done
