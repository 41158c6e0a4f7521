# GPU session: the Python GCM smoke without and with torch loaded, host steps stamped
# (RC_GCM_DEBUG).  Each step bounded; the first failure ends the script.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gcm
make -s -C oracle liboracle.so || exit 3
export RC_GCM_DEBUG=1
NO_TORCH=1 timeout -k 10 60 python -u scripts/gcm_smoke.py > gpurun_out/gcm/smoke_notorch.log 2>&1
rc=$?; echo "smoke (no torch) rc=$rc"; tail -30 gpurun_out/gcm/smoke_notorch.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 60 python -u scripts/gcm_smoke.py > gpurun_out/gcm/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -30 gpurun_out/gcm/smoke.log
exit $rc
