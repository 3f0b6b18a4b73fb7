#!/bin/bash
# Verifier A/B: per variant library (abvar/libgtsfm_hip_<v>.so) the C2 bench under rocprofv3 --stats (RANSAC rows),
# then the product library's verifier / C1 / engine GPU tests.   tools/gpu_ransac_ab.sh TAG v1 v2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; shift
KRE="ransac|normalize" bash tools/gpu_sift_ab.sh $TAG "$@" || exit $?
unset GTSFM_HIP_LIB
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    -k "${K:-verifier or ransac or lund or c4 or all_pairs or frontend or smoke}" > gpurun_out/sab_$TAG/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/sab_$TAG/pytest.log; exit $rc
