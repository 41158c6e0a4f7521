# Large-configuration parity tests and benches (configs 3 ii and 5); each GPU step under its
# own limit, the script stops at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_large.py -x -q > gpurun_out/pytest_large.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_large.log
[ $rc -eq 0 ] || { echo "tests rc=$rc"; exit $rc; }
for c in 3ii 5; do
  timeout -k 10 600 python bench.py --config $c --steps 10 --warmup 2 --cpu-streams 0 > gpurun_out/bench_c$c.log 2>&1
  rc=$?; tail -1 gpurun_out/bench_c$c.log
  [ $rc -eq 0 ] || { echo "bench $c rc=$rc"; exit $rc; }
done
