#!/bin/bash
# attention waves-per-block A/B (SuperGlue tests + C5 grids), then the SIFT PMC passes of the C2 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_r04_gemm.sh aw aw8 || exit $?
bash tools/gpu_pmc_sift.sh r04o || exit $?
