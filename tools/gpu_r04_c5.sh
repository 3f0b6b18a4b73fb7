#!/bin/bash
# C5 kernel timing (kernel-trace stats of a short bench run) plus the SuperGlue GPU tests.   tools/gpu_r04_c5.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r04c5}
timeout -k 10 300 python -u -m pytest tests/test_superglue_gpu.py -q --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_c5 -o run -- python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_c5.json 2> gpurun_out/${TAG}_c5.err
rc=$?; cut -c1-300 gpurun_out/${TAG}_c5.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_c5.err; exit $rc; }
f=$(find gpurun_out/${TAG}_c5 -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/${TAG}_c5_kernel_stats.csv; python tools/kstats.py $f > gpurun_out/${TAG}_c5_ks.txt; head -8 gpurun_out/${TAG}_c5_ks.txt
f=$(find gpurun_out/${TAG}_c5 -name "*kernel_trace.csv" | head -1); python tools/kgrid.py $f sg_ > gpurun_out/${TAG}_c5_grid.txt; head -12 gpurun_out/${TAG}_c5_grid.txt; rm -rf gpurun_out/${TAG}_c5
