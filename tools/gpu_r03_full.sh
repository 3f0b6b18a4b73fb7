#!/bin/bash
# Round-3 full GPU check: GPU suite + smoke + C2 bench with kernel stats (gpu_check.sh), the C4 bench line, then the
# PMC passes (HBM bytes / SQ counters per kernel, the distance GEMM's traffic json, LDS counters).
#   tools/gpu_r03_full.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03}
bash tools/gpu_check.sh $TAG --steps 5 --warmup 2 || exit $?
timeout -k 10 500 python -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${TAG}_c4.json 2> gpurun_out/bench_${TAG}_c4.err
rc=$?; echo "c4 rc=$rc"; cat gpurun_out/bench_${TAG}_c4.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_${TAG}_c4.err; exit $rc; }
bash tools/gpu_pmc_mnn.sh $TAG bench || exit $?
bash tools/gpu_pmc_lds.sh $TAG || exit $?
exit 0
