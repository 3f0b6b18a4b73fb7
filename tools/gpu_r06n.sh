#!/bin/bash
# SuperGlue tests, then the C5 slice line and its per-kernel stats (rocprofv3 --kernel-trace --stats, one step).
#   tools/gpu_r06n.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r06n}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_superglue_gpu.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/${TAG}_pytest.log | head; exit $rc; }
timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_c5.json 2> gpurun_out/${TAG}_c5.err
rc=$?; echo "c5 rc=$rc"; python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['stage_ms'])" gpurun_out/${TAG}_c5.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_c5.err; exit $rc; }
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof -o run -- python -u $R/bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/${TAG}_prof.log 2>&1)
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_prof.log; exit $rc; }
f=$(find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1); python tools/kstats.py $f > gpurun_out/${TAG}_c5_kernels.txt; head -20 gpurun_out/${TAG}_c5_kernels.txt
rm -rf gpurun_out/${TAG}_prof
exit 0
