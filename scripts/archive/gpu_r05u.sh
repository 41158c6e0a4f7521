# Round 5, pass u: the fine tail (RC_TILE_FINE: the launch's last grab per workgroup holds
# one-tile units) -- schedule GPU tests with it, then tile kernel + read probe on one allocation
# for the harness, config 2 and 3 (iii), wave stamps of the harness, pipelined steps.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05u
mkdir -p $out
export TMPDIR=/tmp
RC_TILE_FINE=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_schedule.py tests/test_gpu_parity.py -k "tile_records or random_vs_oracle or group_maxima or harness or constant or fresh or many_small" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -30 $out/pytest.log; exit 3; }
tail -1 $out/pytest.log
timeout -k 10 300 python -u scripts/harness_sched_probe.py harness 6 0:3:0:64:0 0:3:0:64:1 0:3:0:64:2 0:3:0:32:1 > $out/harness.log 2>&1 || { echo "harness probe failed"; tail -5 $out/harness.log; exit 4; }
tail -1 $out/harness.log
RC_LIB_PATH=diag/lib_TSTAMPS.so timeout -k 10 300 python -u scripts/harness_sched_probe.py harness 2 0:3:0:64:0 0:3:0:64:1 > $out/harness_stamps.log 2>&1 || { echo "stamps failed"; tail -5 $out/harness_stamps.log; exit 5; }
tail -1 $out/harness_stamps.log
timeout -k 10 500 python -u scripts/harness_sched_probe.py 2 3 0:3:0:64:0 0:3:0:64:1 0:3:0:64:2 > $out/c2.log 2>&1 || { echo "c2 probe failed"; tail -5 $out/c2.log; exit 6; }
tail -1 $out/c2.log
timeout -k 10 500 python -u scripts/harness_sched_probe.py 3iii 3 0:3:0:64:0 0:3:0:64:1 > $out/c3iii.log 2>&1 || { echo "3iii probe failed"; tail -5 $out/c3iii.log; exit 7; }
tail -1 $out/c3iii.log
timeout -k 10 400 python -u scripts/overlap_ab.py harness 6 p32 p32@0:3:0:64:1 seq seq@0:3:0:64:1 > $out/ab_harness.log 2>&1 || { echo "ab harness failed"; tail -5 $out/ab_harness.log; exit 8; }
tail -1 $out/ab_harness.log
echo done
