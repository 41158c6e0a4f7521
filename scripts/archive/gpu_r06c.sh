set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06c; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_schedule.py tests/test_gpu_lane_chain.py tests/test_gpu_harness.py > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/lib_ab.py 2 4 diag/lib_base6.so diag/lib_sdwa.so > $out/ab_c2.log 2>&1; tail -4 $out/ab_c2.log
timeout -k 10 300 python -u scripts/lib_ab.py 3iii 4 diag/lib_base6.so diag/lib_sdwa.so > $out/ab_3iii.log 2>&1; tail -4 $out/ab_3iii.log
timeout -k 10 300 python -u scripts/lib_ab.py harness 6 diag/lib_base6.so diag/lib_sdwa.so > $out/ab_h.log 2>&1; tail -4 $out/ab_h.log
