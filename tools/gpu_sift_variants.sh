#!/bin/bash
# SIFT kernel times (rocprofv3 --stats over a one-step C2 bench) for the in-tree library and build_var/ variants.
# Usage (through gpurun): tools/gpu_sift_variants.sh [variant ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in base "$@"; do
  if [ $v = base ]; then unset GTSFM_HIP_LIB; else export GTSFM_HIP_LIB=$R/build_var/libgtsfm_hip_$v.so; fi
  echo "== $v"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/sv_$v -o run -- python $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $R/gpurun_out/sv_$v.log 2>&1) || exit 1
  grep -o '"stage_ms": {[^}]*}' $R/gpurun_out/sv_$v.log
  python $R/tools/kstats.py "$(find $R/gpurun_out/sv_$v -name "*kernel_stats.csv" | head -1)" | grep -E "${KPAT:-blur|extrema|descriptor|orientation|refine|topk}"
done
