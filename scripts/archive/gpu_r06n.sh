# round 6: config 3 (iii) pipelined (RC_PIPE_ALL=1) against in sequence and against config 2, on
# one allocation (c2_vs_3iii.py --piped); then bench lines of 3 (iii) both ways, alternating
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06n; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/c2_vs_3iii.py 6 20 --piped > $out/c2_vs_3iii_piped.log 2>&1 || { tail -5 $out/c2_vs_3iii_piped.log; exit 3; }
tail -1 $out/c2_vs_3iii_piped.log
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --config 3iii --steps 20 --cpu-streams 0 > $out/b3iii_seq_$i.log 2>&1 || { tail -5 $out/b3iii_seq_$i.log; exit 4; }
  tail -1 $out/b3iii_seq_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('seq', d['value'], d['ms_per_step'], r['kernel_ms'], r['chain_kernel_ms'], d['pipeline']['pipelined_steps'], d['parity_sha256'])"
  RC_PIPE_ALL=1 timeout -k 10 200 python -u bench.py --config 3iii --steps 20 --cpu-streams 0 > $out/b3iii_pipe_$i.log 2>&1 || { tail -5 $out/b3iii_pipe_$i.log; exit 5; }
  tail -1 $out/b3iii_pipe_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('pipe', d['value'], d['ms_per_step'], r['kernel_ms'], r['chain_kernel_ms'], d['pipeline']['pipelined_steps'], d['parity_sha256'])"
done
