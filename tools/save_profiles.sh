#!/bin/bash
# Copies one gpu_check.sh call's outputs (gpurun_out/*_TAG*) into profiles/ under NAME (e.g. r02c_c2).
TAG=$1; NAME=$2
cd "$(dirname "$0")/.."
cp gpurun_out/bench_${TAG}.json profiles/${NAME}_bench.json
f=$(find gpurun_out/prof_${TAG} -name "*kernel_stats.csv" | sort | tail -n 1)
cp "$f" profiles/${NAME}_kernel_stats.csv
python tools/kstats.py "$f" > profiles/${NAME}_kernel_summary.txt
[ -f gpurun_out/pytest_${TAG}.log ] && cp gpurun_out/pytest_${TAG}.log profiles/${NAME}_pytest_gpu.log
[ -f gpurun_out/smoke_${TAG}.log ] && cp gpurun_out/smoke_${TAG}.log profiles/${NAME}_smoke.log
ls profiles/${NAME}_*
