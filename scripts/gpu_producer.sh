# Producer: GPU parity of the device snapshot producer, then its end-to-end probe.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/producer
export TMPDIR=/tmp
make -s -C oracle liboracle.so || exit 3
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/producer/pytest_pipeline.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/producer/pytest_pipeline.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/producer_probe.py 4096 64 > gpurun_out/producer/64files_4GiB.log 2>&1 || { echo "probe 64 failed"; tail -5 gpurun_out/producer/64files_4GiB.log; exit 4; }
tail -3 gpurun_out/producer/64files_4GiB.log
timeout -k 10 300 python -u scripts/producer_probe.py > gpurun_out/producer/config1_256MiB.log 2>&1 || { echo "probe c1 failed"; tail -5 gpurun_out/producer/config1_256MiB.log; exit 5; }
tail -3 gpurun_out/producer/config1_256MiB.log
