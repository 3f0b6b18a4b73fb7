set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_matcher_gpu.py > gpurun_out/q6_tests.log 2>&1; rc=$?; tail -2 gpurun_out/q6_tests.log; [ $rc -eq 0 ] || exit $rc
GTSFM_MNN=rs timeout -k 10 120 python -u tools/qstamps.py > gpurun_out/q6_stamps.json 2>&1; rc=$?; tail -1 gpurun_out/q6_stamps.json; [ $rc -eq 0 ] || exit $rc
for v in r pp; do
  GTSFM_MNN=$v timeout -k 10 120 python -u tools/matchbench.py 100 > gpurun_out/q6_mb_$v.json 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/q6_mb_$v.json)"
done
