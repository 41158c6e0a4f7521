# Round 4 final validation, part 1: the whole GPU suite, then smoke().
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final4
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/final4/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/final4/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final4/smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/final4/smoke.log; exit 3; }
tail -1 gpurun_out/final4/smoke.log
