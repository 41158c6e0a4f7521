# Lean chain step check: chunker parity tests, then config 3(iii) with the lean step on and off
# (RC_CHAIN_LEAN_OFF=1), then the chain-only PMC of the lean step.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/lean
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_large.py} -m gpu -x -q \
  -p no:cacheprovider --timeout 240 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 $out/pytest.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in on off; do
    if [ $v = off ]; then export RC_CHAIN_LEAN_OFF=1; else unset RC_CHAIN_LEAN_OFF; fi
    timeout -k 10 300 python -u bench.py --config 3iii --cpu-streams 0 > $out/b_${v}_$r.log 2>&1 || { echo "bench $v failed"; tail -n 5 $out/b_${v}_$r.log; exit 4; }
    tail -n 1 $out/b_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v', d['value'], d['ms_per_step'], r['kernel_ms'], r['edge_kernel_ms'], r['chain_kernel_ms'], d['parity_sha256'])"
  done
done
unset RC_CHAIN_LEAN_OFF
REGEX=rc_spec_kernel CFG=3iii bash scripts/gpu_chain_diag.sh > $out/diag.log 2>&1 || { echo diag failed; tail -5 $out/diag.log; exit 5; }
tail -n 20 $out/diag.log
