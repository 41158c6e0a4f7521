# The round-end checks on one box: the whole -m gpu suite, smoke(), and the default bench.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/full
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread --durations=60 > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 $out/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo smoke failed; tail -20 $out/smoke.log; exit 3; }
tail -n 2 $out/smoke.log
timeout -k 10 400 python -u bench.py > $out/bench.log 2>&1 || { echo bench failed; tail -20 $out/bench.log; exit 4; }
tail -n 1 $out/bench.log
