# Round 5, pass z: the group record as one store instruction (lanes 0..2) -- group-record and
# small-window parity tests, then the library before / after on 3 (iii) and config 2.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05z
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_lane_chain.py tests/test_gpu_schedule.py -k "group or lane_chain or full_size or tile_records or random_vs_oracle" > $out/pytest_gstore.log 2>&1 || { echo "tests failed"; tail -30 $out/pytest_gstore.log; exit 3; }
tail -1 $out/pytest_gstore.log
timeout -k 10 400 python -u scripts/lib_ab.py 3iii 4 diag/lib_pre_gstore.so replicat_amd/libreplicat_chunker.so > $out/lib_ab_gstore_3iii.log 2>&1 || { echo "lib ab 3iii failed"; tail -5 $out/lib_ab_gstore_3iii.log; exit 4; }
tail -1 $out/lib_ab_gstore_3iii.log
timeout -k 10 400 python -u scripts/lib_ab.py 2 3 diag/lib_pre_gstore.so replicat_amd/libreplicat_chunker.so > $out/lib_ab_gstore_2.log 2>&1 || { echo "lib ab 2 failed"; tail -5 $out/lib_ab_gstore_2.log; exit 5; }
tail -1 $out/lib_ab_gstore_2.log
echo done
timeout -k 10 400 python -u scripts/lib_ab.py 2 3 diag/lib_NOTAIL_NOXLIST.so replicat_amd/libreplicat_chunker.so > $out/lib_ab_noxlist_2.log 2>&1 || { echo "lib ab noxlist failed"; tail -5 $out/lib_ab_noxlist_2.log; exit 6; }
tail -1 $out/lib_ab_noxlist_2.log
echo done2
