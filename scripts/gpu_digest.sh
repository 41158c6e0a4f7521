# GPU session for the BLAKE2b digests: parity tests, then timing on config 2 and 3(iii).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
make -s -C oracle liboracle.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_digest.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_digest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_digest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python scripts/digest_probe.py 1024 64 > gpurun_out/digest_c2.log 2>&1 || { echo probe failed; tail -20 gpurun_out/digest_c2.log; exit 4; }
tail -1 gpurun_out/digest_c2.log
timeout -k 10 200 python scripts/digest_probe.py 65536 1 2000 80000 > gpurun_out/digest_c3.log 2>&1 || { echo probe3 failed; tail -20 gpurun_out/digest_c3.log; exit 5; }
tail -1 gpurun_out/digest_c3.log
