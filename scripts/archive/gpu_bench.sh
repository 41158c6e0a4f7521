# Quick perf iteration: bench (parity by the in-run config-2 SHA-256) + kernel trace.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-streams 0 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench.log; exit 4; }
tail -1 gpurun_out/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- python3 bench.py --steps 5 --warmup 1 --cpu-streams 0 --no-verify ${BENCH_ARGS:-} > gpurun_out/prof/trace.log 2>&1 || { echo trace failed; tail -20 gpurun_out/prof/trace.log; exit 5; }
python3 scripts/kstats.py
