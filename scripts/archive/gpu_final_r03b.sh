# Round 3, pipelined build: the whole GPU suite + smoke, the default bench line (20 steps, as the
# driver's), then the kernel trace + PMC passes of the default bench command
# (scripts/gpu_profile.sh, last: a profiler failure ends the call there).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/final/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/final/smoke.log; exit 3; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 400 python bench.py --steps 20 > gpurun_out/final/bench.log 2>&1 || { echo bench failed; tail -5 gpurun_out/final/bench.log; exit 3; }
tail -1 gpurun_out/final/bench.log | cut -c1-400
bash scripts/gpu_profile.sh
