#!/bin/bash
# F16_RERANK A/B: the float-matcher / deep GPU tests, then the C3 bench under rocprofv3 stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-c3ab}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "float or superpoint or deep or superglue" > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_${TAG}.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/pytest_${TAG}.log | head; exit $rc; }
bash tools/gpu_prof_cfg.sh ${TAG}_c3 c3 --steps 2 --warmup 1 | head -8
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['stage_ms'], d['verified_rows'], d['pairs_passing_isp'], d['mean_putatives'])" gpurun_out/pc_${TAG}_c3.json
