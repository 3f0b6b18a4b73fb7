#!/bin/bash
# SIFT change check: the SIFT / Lund / engine GPU tests, then the C2 bench under rocprofv3 --stats (SIFT rows)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-sift}
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu -k "sift or lund or all_pairs or frontend or c4 or smoke" tests > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_${TAG}.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/pytest_${TAG}.log | head -20; exit $rc; }
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/p_${TAG} -o run -- python -u $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_c2.json 2> $GRAFT_REPO_ROOT/gpurun_out/${TAG}_c2.err)
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_c2.err; exit $rc; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['stage_ms'])" gpurun_out/${TAG}_c2.json
f=$(find gpurun_out/p_${TAG} -name "*kernel_stats.csv" | head -1); python tools/kstats.py $f | grep -E "blur|extrema|orient|descr"; rm -rf gpurun_out/p_${TAG}
