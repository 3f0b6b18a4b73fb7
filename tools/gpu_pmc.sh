#!/bin/bash
# PMC pass for one workload: gpu_pmc.sh <outname> <counters...> -- <python args...>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$1; shift
CTRS=()
while [ "$1" != "--" ]; do CTRS+=("$1"); shift; done
shift
[ -f gpurun_out/counters_list.txt ] || (cd /tmp && timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters_list.txt 2>&1)
cd /tmp && timeout -k 10 600 rocprofv3 --pmc "${CTRS[@]}" --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT -o run -- python "$GRAFT_REPO_ROOT/$1" "${@:2}" > $GRAFT_REPO_ROOT/gpurun_out/$OUT.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -3 $GRAFT_REPO_ROOT/gpurun_out/$OUT.log
exit $rc
