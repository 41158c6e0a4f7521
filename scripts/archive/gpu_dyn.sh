# Round 3: the tile kernel's dynamic work units.
#   1. chunker GPU parity (parity, lane chain, harness, large, config 4)
#   2. scripts/tile_stamps.py on the new build (diag/lib_TSTAMPS.so): wave end spread
#   3. A/B against the previous build (diag/lib_prev.so): configs 2, 3iii, harness, 3 rounds
#   4. RC_TILE_STATIC / RC_TILE_CHUNK sweep on config 2
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/dyn
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lane_chain.py \
    tests/test_gpu_harness.py tests/test_gpu_large.py tests/test_gpu_config4.py -x -q \
    -p no:cacheprovider --timeout 240 --timeout-method thread > $out/pytest_chunker.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/pytest_chunker.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/tile_stamps.py > $out/tile_stamps.log 2>&1
rc=$?; echo "stamps rc=$rc"; grep '^{' $out/tile_stamps.log | cut -c1-600
[ $rc -eq 0 ] || exit $rc
B=diag/lib_prev.so CONFIGS="2 3iii harness" ROUNDS=3 timeout -k 10 900 bash scripts/gpu_ab.sh > $out/ab.log 2>&1
rc=$?; echo "ab rc=$rc"; cat $out/ab.log
[ $rc -eq 0 ] || exit $rc
for st in 500 750 900; do
  for ck in 16 32 64; do
    RC_TILE_STATIC=$st RC_TILE_CHUNK=$ck timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 \
        --cpu-streams 0 --no-verify > $out/sweep_${st}_${ck}.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "sweep $st $ck rc=$rc"; exit $rc; }
    tail -n 1 $out/sweep_${st}_${ck}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('static', $st, 'chunk', $ck, d['value'], d['ms_per_step'], r['kernel_ms'], r['edge_kernel_ms'], r['chain_kernel_ms'])"
  done
done
exit 0
