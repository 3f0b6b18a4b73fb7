#!/bin/bash
# Bench lines for the variants: C2 with two-view BA, and C4 (1000 images, all 499,500 pairs) at N = 1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r02}
timeout -k 10 300 python -u bench.py --ba --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${TAG}_ba.json 2> gpurun_out/bench_${TAG}_ba.err
rc=$?; echo "bench --ba rc=$rc"; cat gpurun_out/bench_${TAG}_ba.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_${TAG}_ba.err; exit $rc; }
timeout -k 10 600 python -u bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${TAG}_c4.json 2> gpurun_out/bench_${TAG}_c4.err
rc=$?; echo "bench c4 rc=$rc"; cat gpurun_out/bench_${TAG}_c4.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_${TAG}_c4.err; exit $rc; }
