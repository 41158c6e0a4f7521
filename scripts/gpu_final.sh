# Round-end rehearsal plus a kernel-trace profile of the bench command at HEAD.
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_verify.sh || exit $?
mkdir -p gpurun_out/prof_final
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_final/trace -o run -- python3 bench.py --steps 10 --warmup 2 --cpu-streams 0 > gpurun_out/prof_final/trace.log 2>&1 || { echo "trace failed"; tail -n 5 gpurun_out/prof_final/trace.log; exit 5; }
tail -n 1 gpurun_out/prof_final/trace.log
python3 scripts/kstats.py $(find gpurun_out/prof_final/trace -name '*kernel_stats.csv' | head -1)
