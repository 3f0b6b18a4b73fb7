#!/bin/bash
# Round-4 RANSAC call: the verifier / BA GPU tests (E path bit-exact vs the oracle), per-phase solver cycles
# (GTSFM_RANSAC_PROF variant in abvar/), and a kernel trace of the C2 verifier (VGPR / LDS / scratch per kernel).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-"tests/test_verifier_gpu.py tests/test_ba2_gpu.py tests/test_fundamental_gpu.py tests/test_lund_door_c1_gpu.py tests/test_all_pairs_gpu.py tests/test_frontend_batched_gpu.py tests/test_deep_frontend_gpu.py tests/test_c4_gpu.py"}
timeout -k 10 600 python -u -m pytest $T -v --timeout 240 --timeout-method thread > gpurun_out/r04_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r04_tests.log | tail -40; [ $rc -eq 0 ] || exit $rc
[ -n "$SKIP_PROF" ] && exit 0
GTSFM_HIP_LIB=abvar/libgtsfm_hip_prof.so timeout -k 10 300 python -u tools/ransac_prof.py > gpurun_out/r04_ransac_prof.txt 2>&1
rc=$?; tail -25 gpurun_out/r04_ransac_prof.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04_vtrace -o run -- python -u tools/verify_bench.py > gpurun_out/r04_vtrace.log 2>&1
rc=$?; tail -2 gpurun_out/r04_vtrace.log; exit $rc
