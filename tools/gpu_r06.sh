#!/bin/bash
# One GPU call: the given pytest files, then the C2 bench line and the NetVLAD (f3) bench line.
#   tools/gpu_r06.sh TAG "pytest files..."       (run through gpurun; writes gpurun_out/<TAG>_*)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r06}
TESTS=${2:-tests}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest $TESTS -m gpu -x -v -s --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/${TAG}_pytest.log | head -20; exit $rc; }
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err
rc=$?; echo "bench c2 rc=$rc"; cat gpurun_out/${TAG}_c2.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_c2.err; exit $rc; }
timeout -k 10 400 python -u bench.py --config netvlad --steps 3 --warmup 1 > gpurun_out/${TAG}_netvlad.json 2> gpurun_out/${TAG}_netvlad.err
rc=$?; echo "bench netvlad rc=$rc"; cat gpurun_out/${TAG}_netvlad.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_netvlad.err; exit $rc; }
exit 0
