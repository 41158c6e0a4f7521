# GPU session: stateful/keyed BLAKE2b parity + digest regression after the refactor.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_incremental.py tests/test_gpu_digest.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_inc.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_inc.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/digest_probe.py 1024 64 > gpurun_out/digest_c2.log 2>&1 || { echo probe failed; tail -20 gpurun_out/digest_c2.log; exit 4; }
tail -1 gpurun_out/digest_c2.log
