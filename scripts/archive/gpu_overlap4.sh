# Round 3: RC_PIPELINE_END (the last pipelined step's chain on every CU) -- overlap GPU tests,
# then the default bench line at 20 and 5 steps.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/overlap4
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_overlap.py -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $out/pytest.log
[ $rc -eq 0 ] || exit $rc
for k in 20 5; do
  timeout -k 10 300 python -u bench.py --steps $k --cpu-streams 0 > $out/bench_$k.log 2>&1
  rc=$?; echo "bench $k rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  tail -1 $out/bench_$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['pipeline'], d['parity_sha256'])"
done
