# GPU session for the AES-GCM chunk encryption: the watchdog harness on the production kernel, a
# one-message Python smoke, the GCM parity tests, the config-2 probe (digest / derive / encrypt)
# and a rocprofv3 kernel trace of a smaller probe.  Every GPU step has its own time limit; any
# failure ends the script.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gcm
export TMPDIR=/tmp
make -s -C oracle liboracle.so || exit 3
if [ -x diag/gcm_diag_notrace ]; then
  timeout -k 10 60 ./diag/gcm_diag_notrace 10 > gpurun_out/gcm/diag_notrace.log 2>&1
  rc=$?; echo "diag rc=$rc"; tail -4 gpurun_out/gcm/diag_notrace.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 120 python -u scripts/gcm_smoke.py > gpurun_out/gcm/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/gcm/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests/test_gpu_gcm.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gcm/pytest_gcm.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/gcm/pytest_gcm.log
[ $rc -eq 0 ] || exit $rc
if [ "${PROBE:-1}" = 1 ]; then
  timeout -k 10 300 python -u scripts/gcm_probe.py > gpurun_out/gcm/probe_c2.log 2>&1
  rc=$?; echo "probe rc=$rc"; tail -3 gpurun_out/gcm/probe_c2.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gcm/trace -o run -- python3 scripts/gcm_probe.py 256 > gpurun_out/gcm/trace.log 2>&1
  rc=$?; echo "trace rc=$rc"
  find gpurun_out/gcm -name '*kernel_stats.csv'
fi
exit $rc
