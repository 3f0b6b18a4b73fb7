#!/bin/bash
# Per-variant RANSAC kernel times: tools/verify_bench.py under rocprofv3 --kernel-trace --stats for the product library
# and every build_var/libgtsfm_hip_*.so except _old. tools/gpu_vprof.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-vp}
rm -f gpurun_out/verify_ref.npz
GTSFM_HIP_LIB=build_var/libgtsfm_hip_old.so timeout -k 10 300 python -u tools/verify_bench.py > gpurun_out/vp_${TAG}.jsonl 2>&1 || { tail -5 gpurun_out/vp_${TAG}.jsonl; exit 1; }
for so in gtsfm_amd/_lib/libgtsfm_hip.so build_var/libgtsfm_hip_*.so; do
  case $so in *_old.so) continue;; esac
  n=$(basename $so .so)
  GTSFM_HIP_LIB=$so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/vp_${TAG}_$n -o run -- python -u tools/verify_bench.py >> gpurun_out/vp_${TAG}.jsonl 2>&1 || { tail -5 gpurun_out/vp_${TAG}.jsonl; exit 1; }
  rm -rf gpurun_out/vp_${TAG}_$n.keep; echo "== $n"; grep '^{' gpurun_out/vp_${TAG}.jsonl | tail -1 | cut -c1-400
  python tools/kstats.py "$(find gpurun_out/vp_${TAG}_$n -name "*kernel_stats.csv" | head -1)" | grep -i "ransac"
done
exit 0
