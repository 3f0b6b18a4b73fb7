#!/bin/bash
# The other BASELINE configs' bench lines with their CPU baselines.   tools/gpu_lines.sh TAG cfg...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; shift
for cfg in "$@"; do
  timeout -k 10 600 python -u bench.py --config $cfg > gpurun_out/bench_${TAG}_$cfg.json 2> gpurun_out/bench_${TAG}_$cfg.err
  rc=$?; echo "$cfg rc=$rc"; cut -c1-300 gpurun_out/bench_${TAG}_$cfg.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_${TAG}_$cfg.err; exit $rc; }
done
