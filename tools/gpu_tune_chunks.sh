set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_verifier_gpu.py tests/test_all_pairs_gpu.py tests/test_frontend_batched_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r02b.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r02b.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/tune_frontend.py 100 "100,0" "50,0" "45,10" "34,0" "40,20" "25,0" 2>&1 | grep -v amdgpu.ids
