#!/bin/bash
# Kernel-time A/B of one bench config over the product library and build_var/libgtsfm_hip_*.so (except _old):
# tools/gpu_cfg_ab.sh TAG CONFIG [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-ab}; CFG=${2:-c2}; shift 2
for so in gtsfm_amd/_lib/libgtsfm_hip.so build_var/libgtsfm_hip_*.so; do
  case $so in *_old.so) continue;; esac
  [ -f "$so" ] || continue
  n=$(basename $so .so)
  GTSFM_HIP_LIB=$so timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ca_${TAG}_$n -o run -- python -u bench.py --config $CFG --no-cpu-baseline "$@" > gpurun_out/ca_${TAG}_$n.json 2> gpurun_out/ca_${TAG}_$n.err
  rc=$?; echo "== $n rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/ca_${TAG}_$n.err; exit $rc; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d.get('ms_per_step'), d.get('stage_ms'))" gpurun_out/ca_${TAG}_$n.json
  f=$(find gpurun_out/ca_${TAG}_$n -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/ca_${TAG}_$n.csv; rm -rf gpurun_out/ca_${TAG}_$n
  python tools/kstats.py gpurun_out/ca_${TAG}_$n.csv > gpurun_out/ca_${TAG}_$n.txt; sed -n 1,8p gpurun_out/ca_${TAG}_$n.txt
done
