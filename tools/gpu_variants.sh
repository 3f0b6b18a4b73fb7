#!/bin/bash
# matchbench under every build_var/libgtsfm_hip_*.so (GTSFM_HIP_LIB). Usage: gpu_variants.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-v}
for f in build_var/libgtsfm_hip_*.so; do
  n=$(basename $f .so); n=${n#libgtsfm_hip_}
  GTSFM_HIP_LIB=$PWD/$f timeout -k 10 120 python -u tools/matchbench.py 100 > gpurun_out/var_${TAG}_$n.json 2>&1
  rc=$?; echo "$n rc=$rc $(tail -1 gpurun_out/var_${TAG}_$n.json)"; [ $rc -eq 0 ] || exit $rc
done
