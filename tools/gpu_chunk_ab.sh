set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/chunk
for c in 100 25 10 4; do
  timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --resident-chunk $c > gpurun_out/chunk/b$c.json 2> gpurun_out/chunk/b$c.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/chunk/b$c.json'));print($c, d['value'], d['stage_ms'])"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/chunk/prof10" -o run -- python "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --resident-chunk 10 > "$GRAFT_REPO_ROOT/gpurun_out/chunk/prof10.log" 2>&1
