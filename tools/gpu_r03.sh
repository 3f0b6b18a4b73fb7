#!/bin/bash
# Round-3 GPU session: the GPU suite + smoke + C2 bench with rocprof stats (tools/gpu_check.sh), then the C1 / C5 / C3
# bench lines and the RANSAC phase profile. Every GPU step has its own time limit; the call stops at the first failure.
#   tools/gpu_r03.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03}
bash tools/gpu_check.sh $TAG --steps 5 --warmup 2 || exit $?
for cfg in c1 c5 c3; do
  steps=5; [ $cfg = c3 ] && steps=2; [ $cfg = c5 ] && steps=2
  timeout -k 10 400 python -u bench.py --config $cfg --steps $steps --warmup 1 > gpurun_out/bench_${TAG}_$cfg.json 2> gpurun_out/bench_${TAG}_$cfg.err
  rc=$?; echo "$cfg rc=$rc"; cat gpurun_out/bench_${TAG}_$cfg.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_${TAG}_$cfg.err; exit $rc; }
done
# verifier A/B: the product library first (its results are the reference), then every variant in build_var/
[ -d build_var ] || exit 0
timeout -k 10 300 python -u tools/verify_bench.py > gpurun_out/vb_${TAG}.jsonl 2>&1 || { tail -5 gpurun_out/vb_${TAG}.jsonl; exit 1; }
for so in build_var/libgtsfm_hip_*.so; do
  [ -f "$so" ] || continue
  case $so in *prof*) continue;; esac
  GTSFM_HIP_LIB=$so timeout -k 10 300 python -u tools/verify_bench.py >> gpurun_out/vb_${TAG}.jsonl 2>&1 || { tail -5 gpurun_out/vb_${TAG}.jsonl; exit 1; }
done
cat gpurun_out/vb_${TAG}.jsonl
for v in prof prof1; do
  [ -f build_var/libgtsfm_hip_$v.so ] || continue
  GTSFM_HIP_LIB=build_var/libgtsfm_hip_$v.so timeout -k 10 300 python -u tools/ransac_prof.py 100 > gpurun_out/ransac_${v}_${TAG}.txt 2>&1
  rc=$?; echo "ransac $v rc=$rc"; tail -25 gpurun_out/ransac_${v}_${TAG}.txt; [ $rc -eq 0 ] || exit $rc
done
exit 0
