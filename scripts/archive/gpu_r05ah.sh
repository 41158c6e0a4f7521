# Round 5, pass ah: config 3 (iii)'s bench line in sequence (the default policy) and pipelined
# (RC_PIPE_ALL=1), alternated in separate processes on one box, at the driver's 20 steps.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05ah
mkdir -p $out
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --config 3iii --steps 20 --cpu-streams 0 > $out/seq_$i.log 2>&1 || { echo "seq $i failed"; tail -5 $out/seq_$i.log; exit 3; }
  echo "seq $(tail -1 $out/seq_$i.log | cut -c1-200)"
  RC_PIPE_ALL=1 timeout -k 10 300 python -u bench.py --config 3iii --steps 20 --cpu-streams 0 > $out/pipe_$i.log 2>&1 || { echo "pipe $i failed"; tail -5 $out/pipe_$i.log; exit 4; }
  echo "pipe $(tail -1 $out/pipe_$i.log | cut -c1-200)"
done
echo done
