# A subset of the GPU suite, then optionally the default bench line, on one box:
#   bash scripts/gpu_pytest.sh <tag> [--bench] <test files / pytest args...>
# writes gpurun_out/<tag>/pytest.log (and bench.log); stops at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"
tag=$1; shift
bench=0
if [ "${1:-}" = "--bench" ]; then bench=1; shift; fi
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu "$@" > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 $out/pytest.log
[ $rc -eq 0 ] || exit $rc
if [ $bench -eq 1 ]; then
  timeout -k 10 400 python -u bench.py > $out/bench.log 2>&1 || { echo bench failed; tail -20 $out/bench.log; exit 4; }
  tail -n 1 $out/bench.log | cut -c1-300
fi
