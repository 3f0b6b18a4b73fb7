#!/bin/bash
# C3 end-to-end bench (SuperPoint + F16_RERANK) for the in-tree library and build_var/ variants.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in base "$@"; do
  if [ $v = base ]; then unset GTSFM_HIP_LIB; else export GTSFM_HIP_LIB=$GRAFT_REPO_ROOT/build_var/libgtsfm_hip_$v.so; fi
  timeout -k 10 300 python -u bench.py --config ${CFG:-c3} --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${CFG:-c3}_$v.json 2> gpurun_out/${CFG:-c3}_$v.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/${CFG:-c3}_$v.json'));print('$v',d['value'],d['stage_ms_last_step'],d['mean_matches'])"
done
