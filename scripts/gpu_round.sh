# Full GPU session: parity tests, default bench (+calibration), configs, tuning variants.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
make -s -C oracle liboracle.so
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --calibrate > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench.log; exit 4; }
tail -1 gpurun_out/bench.log
bash scripts/gpu_sweep.sh RC_X=0 RC_LIB_PATH=$PWD/diag/lib_IT8.so RC_LIB_PATH=$PWD/diag/lib_IT12.so RC_LIB_PATH=$PWD/diag/lib_PLAIN.so || exit 5
BENCH_ARGS="--calibrate" bash scripts/gpu_sweep.sh RC_LIB_PATH=$PWD/diag/lib_PLAIN.so || exit 6
bash scripts/gpu_configs.sh || exit 7
