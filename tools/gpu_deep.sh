#!/bin/bash
# Deep configs on one GPU call: the C3 and C5 bench lines (with their CPU baselines), then the per-kernel PMC passes
# whose summaries bench.py reads for their roofline "traffic".   tools/gpu_deep.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r04}
for cfg in c3 c5; do
  bash tools/gpu_pmc_deep.sh $TAG $cfg || exit $?
  cp gpurun_out/${TAG}_${cfg}_pmc.json profiles/ || exit 1
  timeout -k 10 500 python -u bench.py --config $cfg --steps 2 --warmup 1 > gpurun_out/bench_${TAG}_$cfg.json 2> gpurun_out/bench_${TAG}_$cfg.err
  rc=$?; echo "$cfg rc=$rc"; cut -c1-300 gpurun_out/bench_${TAG}_$cfg.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_${TAG}_$cfg.err; exit $rc; }
done
