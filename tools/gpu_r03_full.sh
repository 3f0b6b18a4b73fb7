#!/bin/bash
# Round-3 full GPU check: GPU suite + smoke + C2 bench with kernel stats (gpu_check.sh), the C1 / C3 / C4 / C5 bench
# lines, then the PMC passes (HBM bytes / SQ counters per kernel, the distance GEMM's traffic json, LDS counters,
# RANSAC counters). Every GPU step has its own time limit; the call stops at the first failure.
#   tools/gpu_r03_full.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03}
bash tools/gpu_check.sh $TAG --steps 5 --warmup 2 || exit $?
for cfg in c1 c4 c5 c3; do
  steps=5; [ $cfg != c1 ] && steps=2
  timeout -k 10 500 python -u bench.py --config $cfg --steps $steps --warmup 1 > gpurun_out/bench_${TAG}_$cfg.json 2> gpurun_out/bench_${TAG}_$cfg.err
  rc=$?; echo "$cfg rc=$rc"; cut -c1-600 gpurun_out/bench_${TAG}_$cfg.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_${TAG}_$cfg.err; exit $rc; }
done
bash tools/gpu_pmc_mnn.sh $TAG bench || exit $?
bash tools/gpu_pmc_lds.sh $TAG || exit $?
bash tools/gpu_pmc_ransac.sh $TAG || exit $?
exit 0
