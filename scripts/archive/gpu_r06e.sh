# round 6: runner-up group bounds (GroupRecord.second) -- parity, then 3 (iii) pipelined vs in
# sequence on one allocation (overlap_ab, RC_PIPE_ALL=1) and the previous build beside it (lib_ab)
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06e; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_lane_chain.py tests/test_gpu_overlap.py tests/test_gpu_large.py > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
RC_PIPE_ALL=1 timeout -k 10 300 python -u scripts/overlap_ab.py 3iii 4 seq p32 > $out/overlap_3iii.log 2>&1; tail -3 $out/overlap_3iii.log
RC_PIPE_ALL=1 LIB_AB_FLAGS=2 timeout -k 10 300 python -u scripts/lib_ab.py 3iii 4 diag/lib_sdwa.so diag/lib_m2.so > $out/ab_3iii_piped.log 2>&1; tail -1 $out/ab_3iii_piped.log
timeout -k 10 300 python -u scripts/lib_ab.py 3iii 4 diag/lib_sdwa.so diag/lib_m2.so > $out/ab_3iii_seq.log 2>&1; tail -1 $out/ab_3iii_seq.log
