mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_matcher_float_gpu.py > gpurun_out/pytest_fl.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_fl.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/pytest_fl.log | head; exit $rc; }
timeout -k 10 300 python -u tools/sp_matchbench.py 12 || exit 1
timeout -k 10 300 python -u bench.py --config c3 --images 12 --steps 1 --warmup 1 || exit 1
timeout -k 10 300 python -u bench.py --config c5 --images 8 --steps 1 --warmup 1 || exit 1
