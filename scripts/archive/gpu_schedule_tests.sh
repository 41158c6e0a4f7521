# Round 3: the dynamic-schedule parity tests (tests/test_gpu_schedule.py) on this build.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/schedtest
timeout -k 10 900 python -u -m pytest tests/test_gpu_schedule.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/schedtest/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/schedtest/pytest.log
exit $rc
