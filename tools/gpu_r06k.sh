#!/bin/bash
# C3 lines with the matcher certificate (scene-fitted head and the plain seeded head) after the float-matcher tests.
#   tools/gpu_r06k.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r06k}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_matcher_float_gpu.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_c3.json 2> gpurun_out/${TAG}_c3.err
rc=$?; echo "c3 rc=$rc"; python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['stage_ms'], d.get('matcher_certificate'))" gpurun_out/${TAG}_c3.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_c3.err; exit $rc; }
timeout -k 10 500 python -u bench.py --config c3 --c3-head plain --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_c3_plain.json 2> gpurun_out/${TAG}_c3_plain.err
rc=$?; echo "c3 plain rc=$rc"; python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['stage_ms'], d.get('matcher_certificate'))" gpurun_out/${TAG}_c3_plain.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_c3_plain.err; exit $rc; }
exit 0
