# Round 3, third overlap pass (grab counter re-zeroed by the edge kernel, no memset between
# tile kernels; small-window and static-schedule batches in sequence): GPU parity, A/B of the
# reserve on configs 2, 4, 3 (ii), a kernel trace of pipelined and sequential config-2 steps,
# and the default bench line.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/overlap3
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_overlap.py tests/test_gpu_parity.py \
    tests/test_gpu_lane_chain.py tests/test_gpu_schedule.py -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/pytest.log
[ $rc -eq 0 ] || exit $rc
run_ab() {  # log-name config rounds settings...
  local log=$1; shift
  timeout -k 10 300 python -u scripts/overlap_ab.py "$@" > $out/$log.log 2>&1
  local rc=$?; echo "ab $log rc=$rc"; grep '^{' $out/$log.log
  return $rc
}
AB_STEPS=20 run_ab ab_2 2 4 seq p32 p64 && \
AB_STEPS=10 run_ab ab_4 4 3 seq p32 p64 && \
AB_STEPS=20 run_ab ab_3ii 3ii 3 seq p32 p64 || exit 1
AB_STEPS=10 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o run \
    -- python -u scripts/overlap_ab.py 2 1 p32 seq > $out/trace.log 2>&1
rc=$?; echo "trace rc=$rc"
f=$(find $out/trace -name '*kernel_trace.csv' | head -1)
[ -n "$f" ] && python scripts/trace_gaps.py "$f" > $out/gaps.log 2>&1; tail -40 $out/gaps.log
timeout -k 10 300 python -u bench.py --steps 20 > $out/bench_on.log 2>&1
rc=$?; echo "bench on rc=$rc"; tail -c 1200 $out/bench_on.log
exit $rc
