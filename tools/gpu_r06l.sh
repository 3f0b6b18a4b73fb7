#!/bin/bash
# Per-config PMC traffic for C1, then the C2 line with its CPU baseline timed on the whole workload.
#   tools/gpu_r06l.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r06l}
mkdir -p gpurun_out
bash tools/gpu_pmc_mnn.sh $TAG bench c1 > gpurun_out/${TAG}_pmc_c1.log 2>&1
rc=$?; echo "pmc c1 rc=$rc"; tail -3 gpurun_out/${TAG}_pmc_c1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 --cpu-baseline-full > gpurun_out/${TAG}_c2_fullcpu.json 2> gpurun_out/${TAG}_c2_fullcpu.err
rc=$?; echo "c2 rc=$rc"; cat gpurun_out/${TAG}_c2_fullcpu.json | head -c 600; echo; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_c2_fullcpu.err; exit $rc; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['cpu_baseline'])" gpurun_out/${TAG}_c2_fullcpu.json
exit 0
