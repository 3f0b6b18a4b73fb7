#!/bin/bash
# C4 lines (1000 images, all 499,500 pairs) for several pipelined extraction schedules.
#   tools/gpu_r06u.sh TAG "SCHED1 SCHED2 ..."   (bench.py --pipeline values; 0 = off)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r06u}
SCHEDS=${2:-"0"}
mkdir -p gpurun_out
for s in $SCHEDS; do
  timeout -k 10 400 python -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --pipeline $s > gpurun_out/${TAG}_c4_$s.json 2> gpurun_out/${TAG}_c4_$s.err
  rc=$?; echo "c4 pipeline=$s rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_c4_$s.err; exit $rc; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['value_host_to_host'], d['stage_ms'])" gpurun_out/${TAG}_c4_$s.json
done
exit 0
