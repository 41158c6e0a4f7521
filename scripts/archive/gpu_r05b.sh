# Round 5, pass b: the templated tile kernel (per-wave grabs = the round-4 code), the harness's
# workgroup grabs with one and two tile streams, config 2 with two tile streams.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05b
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_schedule.py tests/test_gpu_queue_stream.py tests/test_gpu_overlap.py tests/test_gpu_pipeline.py -k "group or queue or mixed or abandon or g32 or g2 or g256 or g16 or harness" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -30 $out/pytest.log; exit 3; }
tail -2 $out/pytest.log
timeout -k 10 300 python -u scripts/lib_ab.py harness 6 diag/lib_r04.so replicat_amd/libreplicat_chunker.so > $out/lib_ab_harness.log 2>&1 || { echo "lib ab failed"; tail -5 $out/lib_ab_harness.log; exit 6; }
tail -1 $out/lib_ab_harness.log
timeout -k 10 300 python -u scripts/overlap_ab.py harness 6 p32 p32@100:3:0:32 p32x2 p32x2@100:3:0:32 p32x2@100:2:0:32 p32x2@100:4:0:16 > $out/ab_harness.log 2>&1 || { echo "ab harness failed"; tail -5 $out/ab_harness.log; exit 4; }
tail -1 $out/ab_harness.log
timeout -k 10 400 python -u scripts/overlap_ab.py 2 4 p32 p32x2 p32@100:12:128:32 > $out/ab_c2.log 2>&1 || { echo "ab c2 failed"; tail -5 $out/ab_c2.log; exit 5; }
tail -1 $out/ab_c2.log
echo done
