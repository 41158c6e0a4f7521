# One bench line per BASELINE configuration on one box (each under its own time limit; a
# failure ends the script).  The default command first, exactly as the driver runs it.
#   CONFIGS="2 3i 3iii 4 5 3ii harness" bash scripts/gpu_bench_all.sh
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/bench
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > $out/default.log 2>&1 || { echo "default bench failed"; tail -n 5 $out/default.log; exit 4; }
tail -n 1 $out/default.log
for cfg in ${CONFIGS:-3i 3iii 4 5 3ii harness}; do
  extra="--cpu-streams 0"
  [ $cfg = harness ] && extra="--steps 5"
  timeout -k 10 400 python -u bench.py --config $cfg $extra > $out/config_$cfg.log 2>&1 \
    || { echo "bench $cfg failed"; tail -n 5 $out/config_$cfg.log; exit 4; }
  tail -n 1 $out/config_$cfg.log
done
