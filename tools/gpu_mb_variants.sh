#!/bin/bash
# Distance-GEMM microbench over the in-tree library (base) and build_var/ variants (tools/build_variants.sh).
# Usage (through gpurun): tools/gpu_mb_variants.sh [variant ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in base "$@"; do
  if [ $v = base ]; then unset GTSFM_HIP_LIB; else export GTSFM_HIP_LIB=$GRAFT_REPO_ROOT/build_var/libgtsfm_hip_$v.so; fi
  echo "== $v"; timeout -k 10 120 python -u tools/matchbench.py 100 || exit 1
done
