# Profile of the default bench command on one box: rocprofv3 kernel trace + stats, then the PMC
# passes (each counter set in its own run, per MI355X_MICROARCH.md: FETCH_SIZE with the read
# probe for calibration, WRITE_SIZE, SQ sets).  Every GPU step has its own time limit; a failed
# trace ends the script.  Summarise with: python scripts/summarize_profile.py <tag>
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
BENCH="bench.py --steps 5 --warmup 1 --cpu-streams 0 --no-verify"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- python3 $BENCH > gpurun_out/prof/trace.log 2>&1 || { echo trace failed; tail -20 gpurun_out/prof/trace.log; exit 5; }
tail -1 gpurun_out/prof/trace.log
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "rc_tile|rc_read_probe" --output-format csv -d gpurun_out/prof/fetch -o run -- python3 $BENCH --calibrate > gpurun_out/prof/fetch.log 2>&1 || { echo "fetch pass failed rc=$?"; exit 6; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "rc_tile" --output-format csv -d gpurun_out/prof/write -o run -- python3 $BENCH > gpurun_out/prof/write.log 2>&1 || { echo "write pass failed rc=$?"; exit 6; }
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-include-regex "rc_tile" --output-format csv -d gpurun_out/prof/sq -o run -- python3 $BENCH > gpurun_out/prof/sq.log 2>&1 || { echo "sq pass failed rc=$?"; exit 6; }
timeout -s KILL 180 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS --kernel-include-regex "rc_tile" --output-format csv -d gpurun_out/prof/lds -o run -- python3 $BENCH > gpurun_out/prof/lds.log 2>&1 || { echo "lds pass failed rc=$?"; exit 6; }
find gpurun_out/prof -name '*.csv' | head -30
