# round 6: the word before a consecutive tile from the ring (lane 63 of slice 15) instead of a
# load -- parity of the tile paths, then the build against a738351f (diag/lib_a738.so) on one
# allocation: config 2 pipelined, the harness, 3 (iii)
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06q; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_harness.py tests/test_gpu_large.py tests/test_gpu_schedule.py tests/test_gpu_lane_chain.py > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
LIB_AB_FLAGS=2 timeout -k 10 400 python -u scripts/lib_ab.py 2 8 diag/lib_a738.so replicat_amd/libreplicat_chunker.so > $out/ab_c2.log 2>&1 || { tail -5 $out/ab_c2.log; exit 3; }
tail -1 $out/ab_c2.log
LIB_AB_FLAGS=2 timeout -k 10 300 python -u scripts/lib_ab.py harness 12 diag/lib_a738.so replicat_amd/libreplicat_chunker.so > $out/ab_h.log 2>&1 || { tail -5 $out/ab_h.log; exit 4; }
tail -1 $out/ab_h.log
timeout -k 10 400 python -u scripts/lib_ab.py 3iii 6 diag/lib_a738.so replicat_amd/libreplicat_chunker.so > $out/ab_3iii.log 2>&1 || { tail -5 $out/ab_3iii.log; exit 5; }
tail -1 $out/ab_3iii.log
