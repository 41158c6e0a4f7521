# Round 3 final validation (boundary repair, 2-step extensions over 2 x max segments): the whole
# GPU suite + smoke, every configuration's bench line (20 steps), a two-rank rehearsal, then the
# kernel trace + PMC passes of the default bench command (last).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/final/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/final/smoke.log; exit 3; }
tail -1 gpurun_out/final/smoke.log
bash scripts/gpu_final_r03c.sh
