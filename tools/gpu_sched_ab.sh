set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/sched
for v in s2 s4 s8; do
  for r in 0 7; do
    GTSFM_HIP_LIB=$GRAFT_REPO_ROOT/abvar/libgtsfm_hip_$v.so timeout -k 10 300 python -u bench.py --emulate-world 8 --emulate-rank $r --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/sched/${v}_r$r.json 2> gpurun_out/sched/${v}_r$r.err || { tail -5 gpurun_out/sched/${v}_r$r.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('$v r$r', d['ms_per_step'], d['stage_ms'])" gpurun_out/sched/${v}_r$r.json
  done
done
