# Round 3 end: the whole GPU suite + smoke on this build, the default bench line, the kernel
# trace + PMC passes of the default bench command (scripts/gpu_profile.sh), one bench line per
# BASELINE configuration (scripts/gpu_configs.sh), then the allocation spread of the tile kernel
# in three processes (scripts/placement_probe.py, torch allocations).  Two calls (each under
# gpurun's 20-minute limit): `bash scripts/gpu_final_r03.sh tests`, then `... perf`.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final gpurun_out/placement
if [ "${1:-tests}" = tests ]; then
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/final/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/final/smoke.log; exit 3; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/final/bench.log 2>&1 || { echo bench failed; tail -5 gpurun_out/final/bench.log; exit 3; }
tail -1 gpurun_out/final/bench.log
exit 0
fi
bash scripts/gpu_profile.sh || exit $?
bash scripts/gpu_configs.sh || exit $?
for p in 0 1 2; do
  timeout -k 10 300 python -u scripts/placement_probe.py 3 torch > gpurun_out/placement/proc$p.log 2>&1 || { echo "placement $p failed"; tail -5 gpurun_out/placement/proc$p.log; exit 4; }
  grep '^{' gpurun_out/placement/proc$p.log | python3 -c "import json,sys; [print(d['rep'], d['tile_ms'], d['probe_gbs']) for d in map(json.loads, sys.stdin)]"
done
