set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
make -s -C oracle liboracle.so
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; cat gpurun_out/smoke.log | tail -20; exit 3; }
tail -2 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench.log; exit 4; }
tail -3 gpurun_out/bench.log
