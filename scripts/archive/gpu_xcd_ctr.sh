# Round 3: grab counters per XCD (kernels.hip Grabber) -- schedule / parity / overlap GPU tests,
# then the unit-size sweep again (one allocation, scripts/overlap_ab.py).
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/xcd_ctr
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_schedule.py tests/test_gpu_parity.py tests/test_gpu_overlap.py \
    tests/test_gpu_harness.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $out/pytest.log
[ $rc -eq 0 ] || exit $rc
AB_STEPS=20 timeout -k 10 500 python -u scripts/overlap_ab.py 2 4 p32@100:12 p32@100:8 p32@100:6 p32@100:4 p32@0:6 p32@50:4 seq@100:12 seq@100:6 > $out/ab_2.log 2>&1
rc=$?; echo "ab 2 rc=$rc"; grep '^{' $out/ab_2.log
exit $rc
