#!/bin/bash
# One A/B call: per-variant RANSAC kernel times (tools/gpu_vprof.sh), the product's C2 bench under rocprofv3 stats,
# then the SIFT / verifier / engine GPU tests. tools/gpu_ab.sh TAG [pytest -k expr]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-ab}; K=${2:-"sift or lund or verifier or ransac or all_pairs or frontend"}
bash tools/gpu_vprof.sh $TAG || exit $?
rm -rf gpurun_out/vp_${TAG}_*
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_${TAG} -o run -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab_${TAG}.json 2> gpurun_out/ab_${TAG}.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/ab_${TAG}.err; exit $rc; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['stage_ms'])" gpurun_out/ab_${TAG}.json
f=$(find gpurun_out/ab_${TAG} -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/ab_${TAG}_kernel_stats.csv; python tools/kstats.py $f | head -16; rm -rf gpurun_out/ab_${TAG}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_${TAG}.log; exit $rc
