# rocprofv3 kernel trace (+ stats) of one bench command per configuration; each under its own
# time limit, a failure ends the script.   CONFIGS="2 3iii" TAG=r02 bash scripts/gpu_trace.sh
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r02}
for c in ${CONFIGS:-2 3iii}; do
  out=gpurun_out/trace_$c
  mkdir -p $out
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- \
    python3 bench.py --config $c --steps 5 --warmup 1 --cpu-streams 0 ${EXTRA:-} > $out/bench.log 2>&1 \
    || { echo "trace $c failed"; tail -20 $out/bench.log; exit 5; }
  tail -1 $out/bench.log
  f=$(find $out -name '*kernel_stats.csv' | head -1)
  python3 scripts/kstats.py "$f" | tee $out/kstats.txt
done
