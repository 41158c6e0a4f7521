set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python scripts/diag_stamps.py 65536 1 2000 80000 > gpurun_out/stamps_3iii.log 2>&1 || { echo stamps failed; tail gpurun_out/stamps_3iii.log; exit 3; }
cat gpurun_out/stamps_3iii.log
for i in 1 2 3 4; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-streams 0 > gpurun_out/var_$i.log 2>&1 || exit 4
  tail -1 gpurun_out/var_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', d['value'], d['roofline']['kernel_ms'], d['roofline']['chain_kernel_ms'], d['parity_sha256'], d['roofline']['traffic'])"
done
timeout -k 10 300 python bench.py --config 3iii --steps 5 --warmup 1 --cpu-streams 0 > gpurun_out/c3iii.log 2>&1 || exit 5
tail -1 gpurun_out/c3iii.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('3iii', d['value'], d['roofline']['kernel_ms'], d['roofline']['chain_kernel_ms'], d['parity_sha256'])"
