#!/bin/bash
# A/B of the split GEMM's chunk depth / in-flight chunks on the C5 bench (product build + abvar variants).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for so in gtsfm_amd/_lib/libgtsfm_hip.so abvar/libgtsfm_hip_k16s1.so abvar/libgtsfm_hip_k32s1.so abvar/libgtsfm_hip_k32s2.so; do
  n=$(basename $so .so)
  GTSFM_HIP_LIB=$so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/g3_$n -o run -- python -u bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/g3_$n.json 2> gpurun_out/g3_$n.err
  rc=$?; echo "== $n rc=$rc $(cut -c80-140 gpurun_out/g3_$n.json)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/g3_$n.err; exit $rc; }
  f=$(find gpurun_out/g3_$n -name "*kernel_trace.csv" | head -1); python tools/kgrid.py $f sg_gemm3 sg_attention3 | head -6; rm -rf gpurun_out/g3_$n
done
