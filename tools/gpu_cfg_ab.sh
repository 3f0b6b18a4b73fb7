#!/bin/bash
# Bench-config A/B: per variant library (abvar/libgtsfm_hip_<v>.so) one config's bench line under rocprofv3 --stats
# (kernel rows matching KRE), then the product library's GPU tests selected by K.
#   CFG=c3 KRE=fl_ K="matcher_float" tools/gpu_cfg_ab.sh TAG v1 v2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
TAG=$1; shift
mkdir -p gpurun_out/cab_$TAG
for v in "$@"; do
  export GTSFM_HIP_LIB=$R/abvar/libgtsfm_hip_$v.so
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/cab_$TAG/p_$v -o run -- python -u $R/bench.py --config ${CFG:-c2} --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline > $R/gpurun_out/cab_$TAG/$v.json 2> $R/gpurun_out/cab_$TAG/$v.err)
  rc=$?; echo "== $v rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/cab_$TAG/$v.err; exit $rc; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['stage_ms'])" gpurun_out/cab_$TAG/$v.json
  f=$(find gpurun_out/cab_$TAG/p_$v -name "*kernel_stats.csv" | head -1); python tools/kstats.py $f | grep -E "${KRE:-.}" > gpurun_out/cab_$TAG/$v.k; head -12 gpurun_out/cab_$TAG/$v.k; rm -rf gpurun_out/cab_$TAG/p_$v
done
unset GTSFM_HIP_LIB
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$K" > gpurun_out/cab_$TAG/pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/cab_$TAG/pytest.log; exit $rc
fi
