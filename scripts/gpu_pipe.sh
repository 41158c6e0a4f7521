set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
make -s -C oracle liboracle.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_pipe.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_pipe.log
exit $rc
