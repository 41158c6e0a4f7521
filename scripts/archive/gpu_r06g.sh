# round 6: clipped last tiles + cached cursor in rc_tile_kernel<4> -- parity of the small-window
# paths, then lib_ab on 3 (iii) against the SDWA build, in sequence and pipelined
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06g; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_lane_chain.py tests/test_gpu_large.py tests/test_gpu_schedule.py -k "group or lane or 3iii or quad or small or random or digests" > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/lib_ab.py 3iii 6 diag/lib_sdwa.so diag/lib_clip.so > $out/ab_3iii_seq.log 2>&1; tail -1 $out/ab_3iii_seq.log
RC_PIPE_ALL=1 LIB_AB_FLAGS=2 timeout -k 10 300 python -u scripts/lib_ab.py 3iii 4 diag/lib_sdwa.so diag/lib_clip.so > $out/ab_3iii_piped.log 2>&1; tail -1 $out/ab_3iii_piped.log
RC_PIPE_ALL=1 timeout -k 10 300 python -u scripts/overlap_ab.py 3iii 4 seq p32 > $out/overlap_3iii.log 2>&1; tail -1 $out/overlap_3iii.log
