#!/bin/bash
# HBM bytes of the deep configs' kernels (separate rocprofv3 --pmc passes for FETCH_SIZE and WRITE_SIZE over one short
# bench run): gpurun_out/<TAG>_<cfg>_pmc.json, read by bench.py's roofline "traffic" for --config c3 / c5.
#   tools/gpu_pmc_deep.sh TAG c3|c5
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r04}
CFG=${2:-c5}
R=$GRAFT_REPO_ROOT
if [ "$CFG" = c3 ]; then KS="fl_shortlist_kernel,fl_rerank_kernel,conv3_kernel"; else KS="sg_attention3_kernel,sg_gemm3_kernel,sg_gemm_kernel,sk_,conv3_kernel"; fi
dirs=""
for grp in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && timeout -s KILL 600 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc_${TAG}_${CFG}_$grp -o run -- python $R/bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/pmc_${TAG}_${CFG}_$grp.log 2>&1)
  rc=$?; echo "pmc $CFG $grp rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/pmc_${TAG}_${CFG}_$grp.log; exit $rc; }
  dirs="$dirs $R/gpurun_out/pmc_${TAG}_${CFG}_$grp"
done
# steps the profiled command ran: warmup 0 + 1 (host) + 1 (resident) + 2 x 2 instrumented
python $R/tools/pmc_summary.py --json $R/gpurun_out/${TAG}_${CFG}_pmc.json --kernels $KS --steps 6 $dirs && rm -rf $dirs
