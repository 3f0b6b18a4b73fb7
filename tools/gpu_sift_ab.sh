#!/bin/bash
# SIFT kernel A/B: per variant library (abvar/libgtsfm_hip_<v>.so) the C2 bench under rocprofv3 --stats (SIFT rows),
# then FETCH_SIZE per kernel for the variants named in FETCH_VARS.   tools/gpu_sift_ab.sh TAG v1 v2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
TAG=$1; shift
mkdir -p gpurun_out/sab_$TAG
for v in "$@"; do
  export GTSFM_HIP_LIB=$R/${ABDIR:-abvar}/libgtsfm_hip_$v.so
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/sab_$TAG/p_$v -o run -- python -u $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/sab_$TAG/$v.json 2> $R/gpurun_out/sab_$TAG/$v.err)
  rc=$?; echo "== $v rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/sab_$TAG/$v.err; exit $rc; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['stage_ms'])" gpurun_out/sab_$TAG/$v.json
  f=$(find gpurun_out/sab_$TAG/p_$v -name "*kernel_stats.csv" | head -1); python tools/kstats.py $f | grep -E "${KRE:-blur|extrema|orient|descr|topk|refine_k}" > gpurun_out/sab_$TAG/$v.k; cat gpurun_out/sab_$TAG/$v.k; rm -rf gpurun_out/sab_$TAG/p_$v
done
for v in $FETCH_VARS; do
  export GTSFM_HIP_LIB=$R/${ABDIR:-abvar}/libgtsfm_hip_$v.so
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/sab_$TAG/f_$v -o run -- python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/sab_$TAG/f_$v.log 2>&1)
  rc=$?; echo "== fetch $v rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/sab_$TAG/f_$v.log; exit $rc; }
  python tools/pmc_summary.py gpurun_out/sab_$TAG/f_$v | grep -E "blur|extrema|orient|descr" > gpurun_out/sab_$TAG/f_$v.txt; cat gpurun_out/sab_$TAG/f_$v.txt; rm -rf gpurun_out/sab_$TAG/f_$v
done
