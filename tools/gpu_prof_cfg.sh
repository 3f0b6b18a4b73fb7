#!/bin/bash
# rocprofv3 kernel stats of one bench config: tools/gpu_prof_cfg.sh TAG CONFIG [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; CFG=$2; shift 2
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pc_${TAG} -o run -- python -u bench.py --config $CFG --no-cpu-baseline "$@" > gpurun_out/pc_${TAG}.json 2> gpurun_out/pc_${TAG}.err
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pc_${TAG}.err; exit $rc; }
f=$(find gpurun_out/pc_${TAG} -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/pc_${TAG}_kernel_stats.csv; rm -rf gpurun_out/pc_${TAG}
python tools/kstats.py gpurun_out/pc_${TAG}_kernel_stats.csv | head -25
exit 0
