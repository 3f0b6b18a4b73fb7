#!/bin/bash
# Per-rank step times of an emulated N-rank job (bench.py --emulate-world / --emulate-rank).
#   tools/gpu_per_rank.sh TAG "c2:0 c2:7 c4:0 c4:3 c4:7" [N]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/per_rank_$1
N=${3:-8}
for spec in $2; do
  cfg=${spec%%:*}; r=${spec#*:}
  timeout -k 10 400 python -u bench.py --config $cfg --emulate-world $N --emulate-rank $r --steps 3 --warmup 1 --no-cpu-baseline \
      > gpurun_out/per_rank_$1/${cfg}_r$r.json 2> gpurun_out/per_rank_$1/${cfg}_r$r.err || { tail -5 gpurun_out/per_rank_$1/${cfg}_r$r.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('$cfg r$r', d['ms_per_step'], d['stage_ms'])" gpurun_out/per_rank_$1/${cfg}_r$r.json
done
