# Round-end rehearsal: the whole GPU suite, smoke() and the default bench line, each bounded.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/verify
export TMPDIR=/tmp
make -s -C oracle liboracle.so || exit 3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/verify/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/verify/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/verify/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/verify/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/verify/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/verify/bench.log
exit $rc
