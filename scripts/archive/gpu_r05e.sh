# Round 5, pass e: TileRef without padding (no alloca promoted to LDS in the group-grab kernels).
# Parity, then one-allocation A/Bs of per-wave vs workgroup grabs on config 2, 3 (iii), the
# harness, with their read probes; the round-4 library against this one.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05e
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_schedule.py tests/test_gpu_parity.py -k "g32 or g2 or harness or tile_records or random_vs_oracle or group_maxima" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -30 $out/pytest.log; exit 3; }
tail -2 $out/pytest.log
timeout -k 10 400 python -u scripts/harness_sched_probe.py 2 3 100:12:128:0 100:12:0:32 100:6:0:32 100:4:0:64 100:3:0:64 > $out/c2.log 2>&1 || { echo "c2 probe failed"; tail -5 $out/c2.log; exit 6; }
tail -1 $out/c2.log
timeout -k 10 300 python -u scripts/harness_sched_probe.py harness 4 1000:12:128:0 100:2:0:32 100:3:0:64 100:2:0:64 > $out/harness.log 2>&1 || { echo "harness probe failed"; tail -5 $out/harness.log; exit 5; }
tail -1 $out/harness.log
timeout -k 10 400 python -u scripts/lib_ab.py 2 4 diag/lib_r04.so replicat_amd/libreplicat_chunker.so > $out/lib_ab_2.log 2>&1 || { echo "lib ab failed"; tail -5 $out/lib_ab_2.log; exit 4; }
tail -1 $out/lib_ab_2.log
echo done
