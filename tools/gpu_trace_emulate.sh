#!/bin/bash
# rocprofv3 kernel trace of one rank's share (bench.py --emulate-world), then the per-kernel step table.
#   tools/gpu_trace_emulate.sh TAG CONFIG WORLD [RANK]       (through gpurun)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; CFG=$2; N=$3; R=${4:-0}
d=$GRAFT_REPO_ROOT/gpurun_out/tr_${TAG}_${CFG}_w${N}
(cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- \
    python $GRAFT_REPO_ROOT/bench.py --config $CFG --emulate-world $N --emulate-rank $R --steps 2 --warmup 1 \
    > $d.log 2>&1)
rc=$?; echo "trace $CFG w$N rc=$rc"; [ $rc -eq 0 ] || { tail -20 $d.log; exit $rc; }
python tools/step_trace.py "$(find $d -name '*kernel_trace.csv' | head -n 1)" > $d.txt && cat $d.txt
