# Round 5, pass d: the tile scan's 16 lookups batched (sched_barrier) in every tile-kernel
# variant.  Parity of the schedule tests, then one-allocation A/Bs: the round-4 library and the
# pre-fence round-5 library against this one on config 2, 3 (iii) and the harness, and the
# schedules (per-wave / workgroup grabs) with their read probes.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05d
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_schedule.py tests/test_gpu_parity.py -k "g32 or g2 or harness or tile_records or random_vs_oracle or group_maxima" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -30 $out/pytest.log; exit 3; }
tail -2 $out/pytest.log
for c in 2 3iii harness; do
  timeout -k 10 400 python -u scripts/lib_ab.py $c 4 diag/lib_r04.so diag/lib_r05pre.so replicat_amd/libreplicat_chunker.so > $out/lib_ab_$c.log 2>&1 || { echo "lib ab $c failed"; tail -5 $out/lib_ab_$c.log; exit 4; }
  tail -1 $out/lib_ab_$c.log
done
timeout -k 10 400 python -u scripts/harness_sched_probe.py 2 2 100:12:128:0 100:12:0:32 100:6:0:32 100:4:0:64 > $out/c2.log 2>&1 || { echo "c2 probe failed"; tail -5 $out/c2.log; exit 6; }
tail -1 $out/c2.log
timeout -k 10 300 python -u scripts/harness_sched_probe.py harness 4 1000:12:128:0 100:2:0:32 100:3:0:64 100:2:0:64 > $out/harness.log 2>&1 || { echo "harness probe failed"; tail -5 $out/harness.log; exit 5; }
tail -1 $out/harness.log
echo done
