set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_vprof.sh r03s || exit $?
rm -rf gpurun_out/vp_r03s_*
timeout -k 10 300 python -u bench.py --config c1 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_r03s_c1.json 2> gpurun_out/bench_r03s_c1.err
rc=$?; echo "c1 rc=$rc"; python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['stage_ms'], d['verified_rows'], d['pairs_passing_isp'])" gpurun_out/bench_r03s_c1.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "lund or verifier or ransac" > gpurun_out/pytest_r03s.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r03s.log; exit $rc
