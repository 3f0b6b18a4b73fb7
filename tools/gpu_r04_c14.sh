#!/bin/bash
# C1 and C4 bench lines (CPU baselines included).   tools/gpu_r04_c14.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r04h}
for cfg in c1 c4; do
  timeout -k 10 600 python -u bench.py --config $cfg > gpurun_out/bench_${TAG}_$cfg.json 2> gpurun_out/bench_${TAG}_$cfg.err
  rc=$?; echo "$cfg rc=$rc"; cut -c1-400 gpurun_out/bench_${TAG}_$cfg.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_${TAG}_$cfg.err; exit $rc; }
done
