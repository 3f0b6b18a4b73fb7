#!/bin/bash
# A/B of library variants under gtsfm_amd/_lib/var/*: SIFT GPU tests + a short bench stage split per variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in base $(ls gtsfm_amd/_lib/var); do
  if [ $v = base ]; then L=gtsfm_amd/_lib/libgtsfm_hip.so; else L=gtsfm_amd/_lib/var/$v/libgtsfm_hip.so; fi
  GTSFM_HIP_LIB=$PWD/$L timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_sift_gpu.py} -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/var_$v.log 2>&1
  rc=$?; echo "$v tests rc=$rc $(tail -1 gpurun_out/var_$v.log)"; [ $rc -eq 0 ] || exit $rc
  GTSFM_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/var_$v.json 2>gpurun_out/var_$v.err
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/var_$v.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/var_$v.json')); print('$v', d['value'], d['stage_ms'])"
done
