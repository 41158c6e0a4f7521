# Round 3: fewer packets between pipelined tile kernels (no input wait when the caller's stream is
# idle, the timing event doubling as the hand-over event) -- overlap GPU tests, then the A/B
# against the first version's packets on one allocation (scripts/overlap_ab.py, 20 steps).
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/lean
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_overlap.py -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $out/pytest.log
[ $rc -eq 0 ] || exit $rc
AB_STEPS=20 timeout -k 10 300 python -u scripts/overlap_ab.py 2 6 p32 p32:full seq > $out/ab_2.log 2>&1
rc=$?; echo "ab rc=$rc"; grep '^{' $out/ab_2.log
exit $rc
