#!/bin/bash
# Verifier A/B (tools/gpu_vb.sh, no tests) + C2 at 1 / 2 / 3 pair chunks + C4 (chunk overlap of match and verify).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-ov}
bash tools/gpu_vb.sh $TAG none || exit $?
for pc in 0 2475 1650; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --pair-chunk $pc > gpurun_out/bench_${TAG}_pc$pc.json 2> gpurun_out/bench_${TAG}_pc$pc.err
  rc=$?; echo "pc=$pc rc=$rc"; python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['stage_ms'])" gpurun_out/bench_${TAG}_pc$pc.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_${TAG}_pc$pc.err; exit $rc; }
done
timeout -k 10 500 python -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${TAG}_c4.json 2> gpurun_out/bench_${TAG}_c4.err
rc=$?; echo "c4 rc=$rc"; python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['stage_ms'])" gpurun_out/bench_${TAG}_c4.json; exit $rc
