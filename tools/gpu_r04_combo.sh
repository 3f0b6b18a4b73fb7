#!/bin/bash
cd "$GRAFT_REPO_ROOT"
SKIP_PROF= bash tools/gpu_r04_ransac.sh || exit $?
bash tools/gpu_r04_sg.sh r04sg
