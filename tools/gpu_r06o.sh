#!/bin/bash
# SuperGlue tests (DMA-staged GEMM bit-identical to the register-staged one), then the C5 line and per-kernel stats
# for GTSFM_SG_GEMM_DMA = 0 / 2 / 3.
#   tools/gpu_r06o.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r06o}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_superglue_gpu.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/${TAG}_pytest.log | head; exit $rc; }
for v in 0 4; do
  (cd /tmp && export GTSFM_SG_PLANES=$([ $v = 0 ] && echo 0 || echo 1) && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_p$v -o run -- python -u $R/bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/${TAG}_c5_$v.json 2> $R/gpurun_out/${TAG}_c5_$v.err)
  rc=$?; echo "== dma=$v rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_c5_$v.err; exit $rc; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['stage_ms'])" gpurun_out/${TAG}_c5_$v.json
  f=$(find gpurun_out/${TAG}_p$v -name "*kernel_stats.csv" | head -1); python tools/kstats.py $f | grep -E "sg_gemm|attention|sk_pass" > gpurun_out/${TAG}_k$v.txt; cat gpurun_out/${TAG}_k$v.txt
  rm -rf gpurun_out/${TAG}_p$v
done
exit 0
