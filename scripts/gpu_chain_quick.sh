# Chain change, quick check: chunker parity files, then configs 3iii / 2 / 3ii (parity in each line).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/chainq
export TMPDIR=/tmp
make -s -C oracle liboracle.so || exit 3
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/chainq/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 gpurun_out/chainq/pytest.log
[ $rc -eq 0 ] || exit $rc
for cfg in 3iii 2 3ii 3iii; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps 5 --warmup 1 --cpu-streams 0 > gpurun_out/chainq/bench_$cfg.log 2>&1 || { echo "bench $cfg failed"; tail -n 5 gpurun_out/chainq/bench_$cfg.log; exit 4; }
  tail -n 1 gpurun_out/chainq/bench_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$cfg', d['value'], d['ms_per_step'], r['kernel_ms'], r['chain_kernel_ms'], d['parity_sha256'])"
done
for v in ${EDGE_VARIANTS:-}; do
  RC_LIB_PATH=$PWD/diag/lib_$v.so timeout -k 10 300 python -u bench.py --config 3iii --steps 5 --warmup 1 --cpu-streams 0 > gpurun_out/chainq/bench_3iii_$v.log 2>&1 || { echo "bench E$v failed"; exit 5; }
  tail -n 1 gpurun_out/chainq/bench_3iii_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('3iii $v', d['value'], d['ms_per_step'], r['kernel_ms'], r['chain_kernel_ms'], d['parity_sha256'])"
done
