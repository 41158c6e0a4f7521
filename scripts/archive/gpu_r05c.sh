# Round 5, pass c: the simplified group grab (publish at once, config in LDS): GPU schedule
# tests, then per schedule on one allocation the harness's tile kernel, the read probe under the
# same schedule, and (TSTAMPS build) every wave's end; config 2 the same.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05c
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_schedule.py -k "g32 or g2 or g256 or g16 or harness" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -30 $out/pytest.log; exit 3; }
tail -2 $out/pytest.log
S="1000:12:128:0 100:12:0:0 100:4:0:0 100:3:0:32 100:2:0:32 100:3:0:64"
timeout -k 10 300 python -u scripts/harness_sched_probe.py harness 4 $S > $out/harness.log 2>&1 || { echo "harness probe failed"; tail -5 $out/harness.log; exit 4; }
tail -1 $out/harness.log
RC_LIB_PATH=diag/lib_TSTAMPS.so timeout -k 10 300 python -u scripts/harness_sched_probe.py harness 2 $S > $out/harness_stamps.log 2>&1 || { echo "harness stamps failed"; tail -5 $out/harness_stamps.log; exit 5; }
tail -1 $out/harness_stamps.log
timeout -k 10 400 python -u scripts/harness_sched_probe.py 2 2 100:12:128:0 100:12:0:32 100:6:0:32 > $out/c2.log 2>&1 || { echo "c2 probe failed"; tail -5 $out/c2.log; exit 6; }
tail -1 $out/c2.log
echo done
