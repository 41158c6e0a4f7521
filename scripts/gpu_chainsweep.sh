# Chain-kernel variants (diag/ builds) across configs; parity checked by each bench run.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -k "segmented or golden or random or open or digests" > gpurun_out/pytest_chain.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_chain.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/chainsweep.log
for cfg in ${CONFIGS:-3iii 2 4}; do
  for lib in default ${LIBS:-}; do
    if [ $lib = default ]; then envs="RC_X=0"; else envs="RC_LIB_PATH=$PWD/diag/lib_$lib.so"; fi
    env $envs timeout -k 10 300 python bench.py --config $cfg --steps 5 --warmup 1 --cpu-streams 0 >> gpurun_out/chainsweep.log 2>&1 || { echo "failed $cfg $lib"; exit 4; }
    tail -1 gpurun_out/chainsweep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', '$lib', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['chain_kernel_ms'], d['parity_sha256'])"
  done
done
