#!/bin/bash
# Per-rank lines: rank R's share of an N-rank job on one GPU (bench.py --emulate-world), for each N given.
#   tools/gpu_emulate.sh TAG CONFIG RANK N...      (through gpurun; writes gpurun_out/emu_TAG_CONFIG_wN_rR.json)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; CFG=$2; RANK=$3; shift 3
for N in "$@"; do
  out=gpurun_out/emu_${TAG}_${CFG}_w${N}_r${RANK}
  timeout -k 10 600 python -u bench.py --config $CFG --emulate-world $N --emulate-rank $RANK --steps 5 --warmup 2 \
      > $out.json 2> $out.err
  rc=$?; echo "$CFG N=$N rank $RANK rc=$rc"; cut -c1-400 $out.json; [ $rc -eq 0 ] || { tail -20 $out.err; exit $rc; }
done
