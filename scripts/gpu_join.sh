# Segmented-chain parity (parallel join and sequential walk), large configs, then config 3 (ii)
# bench + kernel trace.  Stops at the first failing step.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -x -q -k "segmented or large or split or config" > gpurun_out/pytest_join.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_join.log; [ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--config 3ii" bash scripts/gpu_bench.sh
