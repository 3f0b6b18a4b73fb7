#!/bin/bash
# SuperGlue GEMM tile A/B: product (tests + C5 bench + kernel grid), then the C5 kernel grid of abvar/libgtsfm_hip_<v>.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-gemm}; shift
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_superglue_gpu.py tests/test_deep_frontend_gpu.py > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_${TAG}.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_${TAG}.log | head -20; exit $rc; }
for v in prod "$@"; do
  if [ $v != prod ]; then export GTSFM_HIP_LIB=$GRAFT_REPO_ROOT/abvar/libgtsfm_hip_$v.so; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_$v -o run -- python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_${v}_c5.json 2> gpurun_out/${TAG}_${v}_c5.err
  rc=$?; echo "== $v rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_${v}_c5.err; exit $rc; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['stage_ms'], d['roofline']['frac'])" gpurun_out/${TAG}_${v}_c5.json
  f=$(find gpurun_out/${TAG}_$v -name "*kernel_trace.csv" | head -1); python tools/kgrid.py $f sg_ sk_ > gpurun_out/${TAG}_${v}_grid.txt; head -12 gpurun_out/${TAG}_${v}_grid.txt; rm -rf gpurun_out/${TAG}_$v
done
