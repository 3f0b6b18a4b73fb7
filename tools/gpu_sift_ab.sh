#!/bin/bash
# SIFT A/B: C2 bench extract time + kernel stats for the product library and build_var/libgtsfm_hip_*.so (except
# _old), then the SIFT GPU tests. tools/gpu_sift_ab.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-sa}
for so in gtsfm_amd/_lib/libgtsfm_hip.so build_var/libgtsfm_hip_*.so; do
  case $so in *_old.so) continue;; esac
  n=$(basename $so .so)
  GTSFM_HIP_LIB=$so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sa_${TAG}_$n -o run -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sa_${TAG}_$n.json 2> gpurun_out/sa_${TAG}_$n.err
  rc=$?; echo "== $n rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/sa_${TAG}_$n.err; exit $rc; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['stage_ms'], d['verified_rows'], d['pairs_passing_isp'], d['mean_putatives'])" gpurun_out/sa_${TAG}_$n.json
  f=$(find gpurun_out/sa_${TAG}_$n -name "*kernel_stats.csv" | head -1); python tools/kstats.py $f | grep -v ransac | head -14; cp $f gpurun_out/sa_${TAG}_$n.csv; rm -rf gpurun_out/sa_${TAG}_$n
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "sift or lund or smoke or frontend" > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_${TAG}.log; exit $rc
