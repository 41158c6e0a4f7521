# GPU session: parity tests, bench, rocprofv3 kernel trace + PMC passes.  Every GPU step has
# its own time limit; a fault/abort/timeout ends the script (pytest failures do not).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TAG=${TAG:-r01}
make -s -C oracle liboracle.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench.log; exit 4; }
tail -1 gpurun_out/bench.log
BENCH="bench.py --steps 5 --warmup 1 --cpu-streams 0 --no-verify"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- python3 $BENCH > gpurun_out/prof/trace.log 2>&1 || { echo trace failed; tail -20 gpurun_out/prof/trace.log; exit 5; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/fetch -o run -- python3 $BENCH --calibrate > gpurun_out/prof/fetch.log 2>&1 || echo "fetch pass failed rc=$?"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/write -o run -- python3 $BENCH > gpurun_out/prof/write.log 2>&1 || echo "write pass failed rc=$?"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/prof/sq -o run -- python3 $BENCH > gpurun_out/prof/sq.log 2>&1 || echo "sq pass failed rc=$?"
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/prof/lds -o run -- python3 $BENCH > gpurun_out/prof/lds.log 2>&1 || echo "lds pass failed rc=$?"
find gpurun_out/prof -name '*.csv' | head -30
