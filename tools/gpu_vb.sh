#!/bin/bash
# Verifier A/B: build_var/libgtsfm_hip_old.so (reference results) then the product library (with a rocprofv3 kernel
# trace), then the verifier / engine GPU tests. tools/gpu_vb.sh TAG [pytest -k expr | none]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-vb}; K=${2:-"verifier or ransac or lund or all_pairs or frontend"}
rm -f gpurun_out/verify_ref.npz
GTSFM_HIP_LIB=build_var/libgtsfm_hip_old.so timeout -k 10 300 python -u tools/verify_bench.py > gpurun_out/vb_${TAG}.jsonl 2>&1 || { tail -5 gpurun_out/vb_${TAG}.jsonl; exit 1; }
for so in build_var/libgtsfm_hip_*.so; do
  case $so in *_old.so) continue;; esac
  GTSFM_HIP_LIB=$so timeout -k 10 300 python -u tools/verify_bench.py >> gpurun_out/vb_${TAG}.jsonl 2>&1 || { tail -5 gpurun_out/vb_${TAG}.jsonl; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/vbprof_${TAG} -o run -- python -u tools/verify_bench.py >> gpurun_out/vb_${TAG}.jsonl 2>&1 || { tail -5 gpurun_out/vb_${TAG}.jsonl; exit 1; }
grep '^{' gpurun_out/vb_${TAG}.jsonl
python tools/kstats.py "$(find gpurun_out/vbprof_${TAG} -name "*kernel_stats.csv" | sort | tail -n 1)" | grep -i "ransac\|mnn_pp"
[ "$K" = none ] && exit 0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_${TAG}.log; exit $rc
