set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest ${1:-tests/test_superglue_gpu.py} -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_sg.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert" gpurun_out/pytest_sg.log | head -30; tail -3 gpurun_out/pytest_sg.log; exit $rc
