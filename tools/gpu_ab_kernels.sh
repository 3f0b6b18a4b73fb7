#!/bin/bash
# A/B of library variants ($ABDIR/libgtsfm_hip_<v>.so) on one bench command: per variant the rocprofv3 kernel
# stats of the command, filtered by PATTERN.   ABDIR=build_ab tools/gpu_ab_kernels.sh TAG "PATTERN" "BENCH ARGS" v1 v2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
TAG=$1; PAT=$2; ARGS=$3; shift 3
mkdir -p gpurun_out/ab_$TAG
for v in "$@"; do
  export GTSFM_HIP_LIB=$R/${ABDIR:-build_ab}/libgtsfm_hip_$v.so
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ab_$TAG/p_$v -o run -- python -u $R/bench.py $ARGS > $R/gpurun_out/ab_$TAG/$v.json 2> $R/gpurun_out/ab_$TAG/$v.err)
  rc=$?; echo "== $v rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/ab_$TAG/$v.err; exit $rc; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['stage_ms'])" gpurun_out/ab_$TAG/$v.json
  f=$(find gpurun_out/ab_$TAG/p_$v -name "*kernel_stats.csv" | head -1); python tools/kstats.py $f | grep -E "$PAT" > gpurun_out/ab_$TAG/$v.k; cat gpurun_out/ab_$TAG/$v.k; rm -rf gpurun_out/ab_$TAG/p_$v
done
