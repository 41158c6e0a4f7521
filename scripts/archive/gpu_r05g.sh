# Round 5, pass g (after the container was re-created): where HEAD stands.  Schedule + parity
# tests of the workgroup grabs, the harness's schedules with their read probes (plain and wave
# stamps), the round-4 library against HEAD on the harness and config 2, then the harness and
# default bench lines.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05g
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_schedule.py tests/test_gpu_parity.py -k "g32 or g2 or harness or tile_records or random_vs_oracle or group_maxima" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -30 $out/pytest.log; exit 3; }
tail -2 $out/pytest.log
S="1000:12:128:0 100:3:0:64 0:3:0:64 100:2:0:32 100:2:0:128 0:2:0:64"
timeout -k 10 300 python -u scripts/harness_sched_probe.py harness 4 $S > $out/harness.log 2>&1 || { echo "harness probe failed"; tail -5 $out/harness.log; exit 4; }
tail -1 $out/harness.log
RC_LIB_PATH=diag/lib_TSTAMPS.so timeout -k 10 300 python -u scripts/harness_sched_probe.py harness 2 1000:12:128:0 100:3:0:64 0:3:0:64 > $out/harness_stamps.log 2>&1 || { echo "harness stamps failed"; tail -5 $out/harness_stamps.log; exit 5; }
tail -1 $out/harness_stamps.log
timeout -k 10 300 python -u scripts/lib_ab.py harness 6 diag/lib_r04.so replicat_amd/libreplicat_chunker.so > $out/lib_ab_harness.log 2>&1 || { echo "lib ab failed"; tail -5 $out/lib_ab_harness.log; exit 6; }
tail -1 $out/lib_ab_harness.log
timeout -k 10 400 python -u scripts/lib_ab.py 2 4 diag/lib_r04.so replicat_amd/libreplicat_chunker.so > $out/lib_ab_2.log 2>&1 || { echo "lib ab 2 failed"; tail -5 $out/lib_ab_2.log; exit 7; }
tail -1 $out/lib_ab_2.log
timeout -k 10 300 python -u bench.py --config harness --steps 20 --warmup 3 > $out/bench_harness.log 2>&1 || { echo "bench harness failed"; tail -5 $out/bench_harness.log; exit 8; }
tail -1 $out/bench_harness.log | cut -c1-600
timeout -k 10 400 python -u bench.py > $out/bench.log 2>&1 || { echo "bench failed"; tail -5 $out/bench.log; exit 9; }
tail -1 $out/bench.log | cut -c1-600
echo done
