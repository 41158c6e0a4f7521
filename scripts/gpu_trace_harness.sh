# Kernel trace of the reference-harness workload (one 5.12 GB stream: segment-parallel chain).
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/trace_harness
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- \
  python3 bench.py --config harness --steps 5 --warmup 1 --cpu-streams 0 --no-verify > $out/bench.log 2>&1 \
  || { echo "trace failed"; tail -n 20 $out/bench.log; exit 5; }
tail -n 1 $out/bench.log | cut -c1-400
python3 scripts/kstats.py "$(find $out -name '*kernel_stats.csv' | head -1)" | tee $out/kstats.txt
