# Round 3: repair + lists skipped by a long extension (scan kernel's entry recurrence) --
# chunker GPU parity, then the segment floor / extension sweep (scripts/chain_ab.py).
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/repair3
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_harness.py \
    tests/test_gpu_large.py tests/test_gpu_config4.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $out/pytest.log
[ $rc -eq 0 ] || exit $rc
run() {  # log config settings...
  local log=$1; shift
  timeout -k 10 300 python -u scripts/chain_ab.py "$@" > $out/$log.log 2>&1
  local rc=$?; echo "ab $log rc=$rc"; grep '^{' $out/$log.log
  return $rc
}
M=5120000
run harness harness 4 f3:4 f2:2 f2:1 f1:2 f1:1 $M:1 && \
run 3ii 3ii 4 0:4 0:2 0:1 && \
run c4 4 3 0:4 0:2 0:1 && \
run c2 2 3 0:4 0:2 0:1
