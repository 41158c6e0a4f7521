# Round 5, first pass: workgroup grabs (RC_TILE_GROUP) -- the schedule's GPU parity tests, then
# one-allocation A/Bs of the harness and config 2 against the per-wave grabs, the round-4 library
# against this one (per-wave grabs: the refactor must not cost), and wave end stamps.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05a
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_schedule.py > $out/pytest_schedule.log 2>&1 || { echo "schedule tests failed"; tail -30 $out/pytest_schedule.log; exit 3; }
tail -2 $out/pytest_schedule.log
timeout -k 10 300 python -u scripts/overlap_ab.py harness 6 p32 p32@100:12:0:0 p32@100:4:0:32 p32@100:3:0:32 p32@100:2:0:32 p32@0:2:0:64 seq p32@100:2:0:16 > $out/ab_harness.log 2>&1 || { echo "ab harness failed"; tail -5 $out/ab_harness.log; exit 4; }
tail -1 $out/ab_harness.log
timeout -k 10 400 python -u scripts/overlap_ab.py 2 4 p32 p32@100:6:0:32 p32@100:4:0:32 p32@100:3:0:64 p32@100:8:0:16 > $out/ab_c2.log 2>&1 || { echo "ab c2 failed"; tail -5 $out/ab_c2.log; exit 5; }
tail -1 $out/ab_c2.log
timeout -k 10 300 python -u scripts/lib_ab.py harness 6 diag/lib_r04.so replicat_amd/libreplicat_chunker.so > $out/lib_ab_harness.log 2>&1 || { echo "lib ab failed"; tail -5 $out/lib_ab_harness.log; exit 6; }
tail -1 $out/lib_ab_harness.log
RC_TILE_DYN_MIN=0 RC_TILE_CHUNK=2 RC_TILE_GROUP=32 timeout -k 10 300 python -u scripts/tile_stamps.py harness > $out/stamps_harness_g32.log 2>&1 || { echo "stamps failed"; tail -5 $out/stamps_harness_g32.log; exit 7; }
grep '^{' $out/stamps_harness_g32.log | cut -c1-400
echo done
