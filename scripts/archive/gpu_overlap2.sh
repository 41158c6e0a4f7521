# Round 3, second overlap pass (profiles/r03/overlap/pass2): 32- and 64-CU reserves on configs 2,
# 4, 3 (ii), the harness and 3 (iii), the wall clock without per-call events, and a kernel trace
# of pipelined config-2 steps (gaps between tile kernels on the tile queue).  (Run then with
# RC_PIPE_GROUPS=1 for 3 iii, since renamed RC_PIPE_ALL.)
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/overlap2
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_overlap.py -x -v -p no:cacheprovider \
    --timeout 300 --timeout-method thread > $out/pytest_overlap.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/pytest_overlap.log
[ $rc -eq 0 ] || exit $rc
run_ab() {  # log-name config settings...
  local log=$1; shift
  timeout -k 10 300 python -u scripts/overlap_ab.py "$@" > $out/$log.log 2>&1
  local rc=$?; echo "ab $log rc=$rc"; grep '^{' $out/$log.log
  return $rc
}
run_ab ab_2 2 4 seq p32 p64 && \
AB_TIMING=0 run_ab ab_2_notiming 2 4 seq p32 && \
RC_PIPE_ALL=1 run_ab ab_harness harness 4 seq p32 p64 && \
run_ab ab_4 4 3 seq p32 && \
run_ab ab_3ii 3ii 3 seq p32 && \
RC_PIPE_ALL=1 run_ab ab_3iii 3iii 3 seq p32 || exit 1
AB_STEPS=10 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o run \
    -- python -u scripts/overlap_ab.py 2 1 p32 > $out/trace.log 2>&1
rc=$?; echo "trace rc=$rc"
f=$(find $out/trace -name '*kernel_trace.csv' | head -1)
python scripts/trace_gaps.py "$f" > $out/gaps.log 2>&1; tail -30 $out/gaps.log
exit 0
