#!/bin/bash
# Pipelined front-end schedule: its GPU tests, then C2 lines for several extraction-chunk schedules.
#   tools/gpu_r06t.sh TAG "SCHED1 SCHED2 ..."   (each schedule as bench.py --pipeline takes it; 0 = off)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r06t}
SCHEDS=${2:-"0 50"}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_all_pairs_gpu.py -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/${TAG}_pytest.log | head; exit $rc; }
for s in $SCHEDS; do
  timeout -k 10 300 python -u bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline --pipeline $s > gpurun_out/${TAG}_c2_$s.json 2> gpurun_out/${TAG}_c2_$s.err
  rc=$?; echo "c2 pipeline=$s rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_c2_$s.err; exit $rc; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['value_host_to_host'], d['stage_ms'])" gpurun_out/${TAG}_c2_$s.json
done
exit 0
