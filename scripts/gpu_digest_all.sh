# BLAKE2b change check: every test that runs a BLAKE2b kernel, then the digest timings.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/digest
export TMPDIR=/tmp
make -s -C oracle liboracle.so || exit 3
timeout -k 10 500 python -u -m pytest tests/test_gpu_digest.py tests/test_gpu_incremental.py tests/test_gpu_pipeline.py tests/test_gpu_gcm.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/digest/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/digest/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/digest_probe.py 1024 64 > gpurun_out/digest/digest_c2.log 2>&1 || { echo probe failed; tail -20 gpurun_out/digest/digest_c2.log; exit 4; }
tail -1 gpurun_out/digest/digest_c2.log
timeout -k 10 200 python scripts/digest_probe.py 65536 1 2000 80000 > gpurun_out/digest/digest_c3.log 2>&1 || { echo probe3 failed; tail -20 gpurun_out/digest/digest_c3.log; exit 5; }
tail -1 gpurun_out/digest/digest_c3.log
