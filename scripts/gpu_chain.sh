# Chain iteration: parity subset, per-step stamps on config 3 (iii), benches of 3iii and 2.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -x -q -k "segmented or golden or random or open or digests or split or config3ii" > gpurun_out/pytest_chain.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_chain.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/diag_stamps.py 65536 1 2000 80000 > gpurun_out/stamps_3iii.log 2>&1 || { echo stamps failed; tail gpurun_out/stamps_3iii.log; exit 3; }
tail -5 gpurun_out/stamps_3iii.log
for cfg in 3iii 2 ${MORE:-}; do
  timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 2 --cpu-streams 0 > gpurun_out/c$cfg.log 2>&1 || exit 5
  tail -1 gpurun_out/c$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', d['value'], d['roofline']['kernel_ms'], d['roofline']['chain_kernel_ms'], d['parity_sha256'])"
done
