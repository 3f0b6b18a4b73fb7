#!/bin/bash
# Environment A/B of the product library: per variant NAME=VAR=VALUE, the C2 bench under rocprofv3 --stats (kernel
# rows matching $KRE, default the SIFT kernels); several assignments per variant joined by commas.
#   tools/gpu_env_ab.sh TAG off=GTSFM_BLUR_STREAM=0 s6=GTSFM_BLUR_STREAM=1,GTSFM_BLUR_SEGS=6
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
TAG=$1; shift
KRE=${KRE:-"blur|extrema|orient|descr|topk|refine_k"}
mkdir -p gpurun_out/eab_$TAG
for spec in "$@"; do
  v=${spec%%=*}; assign=${spec#*=}
  (cd /tmp && for a in ${assign//,/ }; do export "$a"; done && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/eab_$TAG/p_$v -o run -- python -u $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $R/gpurun_out/eab_$TAG/$v.json 2> $R/gpurun_out/eab_$TAG/$v.err)
  rc=$?; echo "== $v ($assign) rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/eab_$TAG/$v.err; exit $rc; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['stage_ms'])" gpurun_out/eab_$TAG/$v.json
  f=$(find gpurun_out/eab_$TAG/p_$v -name "*kernel_stats.csv" | head -1); python tools/kstats.py $f | grep -E "$KRE" > gpurun_out/eab_$TAG/$v.k; cat gpurun_out/eab_$TAG/$v.k
  rm -rf gpurun_out/eab_$TAG/p_$v
done
