#!/bin/bash
# SIFT diagnostics: FETCH_SIZE calibration of the row-walk micro-benchmark (4 / 8 / 16-byte loads of a known byte
# count), then tools/gpu_sift_ab.sh over the build_var variants. tools/gpu_sift_diag.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-sd}
timeout -k 10 120 ./build_var/rowwalk > gpurun_out/rw_${TAG}.txt 2>&1 || exit $?
cat gpurun_out/rw_${TAG}.txt
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/rwp_${TAG} -o run -- ./build_var/rowwalk > /dev/null 2>&1 || exit $?
f=$(find gpurun_out/rwp_${TAG} -name "*counter_collection.csv" | head -1)
python - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    acc[r['Kernel_Name'][:40]].append(float(r['Counter_Value']))
for k, v in acc.items():
    print('%-40s launches %d  FETCH_SIZE %.3f GB per launch (x1024 B)' % (k, len(v), sum(v) / len(v) * 1024 / 1e9))
PY
rm -rf gpurun_out/rwp_${TAG}
bash tools/gpu_sift_ab.sh ${TAG}
