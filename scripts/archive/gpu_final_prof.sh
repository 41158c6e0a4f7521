# Round 3: the whole GPU suite on this build, then the kernel trace + PMC passes of the default
# bench command (scripts/gpu_profile.sh), one bench line per BASELINE configuration
# (scripts/gpu_configs.sh), then the harness schedule sweep.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/final/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_profile.sh || exit $?
bash scripts/gpu_configs.sh || exit $?
mkdir -p gpurun_out/sched
timeout -k 10 300 python -u scripts/tile_sched_ab.py harness 6 1000:32 0:32 0:16 0:8 250:8 > gpurun_out/sched/ab_harness2.log 2>&1
rc=$?; echo "harness sched rc=$rc"; grep '^{' gpurun_out/sched/ab_harness2.log
exit $rc
