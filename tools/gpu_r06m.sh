#!/bin/bash
# SuperGlue tests (fused one-pass Sinkhorn vs the goldens and vs the two-pass form), then the C5 slice line with the
# fused pass and with the two-pass form (GTSFM_SG_SINKHORN_TWO_PASS=1).
#   tools/gpu_r06m.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r06m}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_superglue_gpu.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/${TAG}_pytest.log | head; exit $rc; }
for v in fused two; do
  if [ $v = two ]; then export GTSFM_SG_SINKHORN_TWO_PASS=1; else unset GTSFM_SG_SINKHORN_TWO_PASS; fi
  timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_c5_$v.json 2> gpurun_out/${TAG}_c5_$v.err
  rc=$?; echo "c5 $v rc=$rc"; python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['stage_ms'])" gpurun_out/${TAG}_c5_$v.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_c5_$v.err; exit $rc; }
done
exit 0
