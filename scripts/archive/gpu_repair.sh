# Round 3: boundary repair in the merge kernel -- chunker GPU parity (segmented chains in the
# three join modes, the harness at forced short segments), then the chain phase of the harness
# and config 3 (ii) under shorter segments / fewer extension steps, with and without repair.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/repair
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_harness.py \
    tests/test_gpu_large.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $out/pytest.log
[ $rc -eq 0 ] || exit $rc
M=5120000
timeout -k 10 300 python -u scripts/chain_ab.py harness 4 0:4 0:4:norepair $((3*M)):2 $((3*M)):1 $((2*M)):2 $((2*M)):1 $M:2 $M:1 $M:1:norepair > $out/ab_harness.log 2>&1
rc=$?; echo "ab harness rc=$rc"; grep '^{' $out/ab_harness.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/chain_ab.py 3ii 4 0:4 $((2*M)):2 $((2*M)):1 $M:2 $M:1 > $out/ab_3ii.log 2>&1
rc=$?; echo "ab 3ii rc=$rc"; grep '^{' $out/ab_3ii.log
exit $rc
