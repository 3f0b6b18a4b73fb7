#!/bin/bash
# C3 end-to-end bench line + rocprofv3 kernel stats of the C3 and C5 benches (SuperPoint conv_mfma, SuperGlue
# sg_attention / sg_gemm, F16_RERANK). Usage (through gpurun): tools/gpu_dl_prof.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-dl}
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --config c3 --steps 1 --warmup 1 > gpurun_out/bench_${TAG}_c3.json 2> gpurun_out/bench_${TAG}_c3.err
rc=$?; echo "c3 rc=$rc"; cat gpurun_out/bench_${TAG}_c3.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_${TAG}_c3.err; exit $rc; }
timeout -k 10 300 python -u bench.py --config c5 --steps 2 --warmup 1 > gpurun_out/bench_${TAG}_c5.json 2> gpurun_out/bench_${TAG}_c5.err
rc=$?; echo "c5 rc=$rc"; cat gpurun_out/bench_${TAG}_c5.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_${TAG}_c5.err; exit $rc; }
for C in c5 c3; do
  if [ $C = c3 ]; then EXTRA="--images 24"; else EXTRA=""; fi
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_$C" \
      -o run -- python "$GRAFT_REPO_ROOT/bench.py" --config $C --steps 1 --warmup 1 $EXTRA > "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_$C.log" 2>&1
  rc=$?; cd "$GRAFT_REPO_ROOT"; echo "prof $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python tools/kstats.py "$(find gpurun_out/prof_${TAG}_$C -name "*kernel_stats.csv" | sort | tail -n 1)" | head -14
done
exit 0
