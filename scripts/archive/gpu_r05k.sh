# Round 5, pass k: the edge kernel's coalesced tie-count scan -- tie-tile parity tests, then the
# library before / after on config 2, 3 (iii) and the harness (sequential calls: edge_ms).
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05k
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_schedule.py -k "tile_records or constant or random_vs_oracle or group_maxima" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -30 $out/pytest.log; exit 3; }
tail -2 $out/pytest.log
for c in 2 3iii harness; do
  timeout -k 10 400 python -u scripts/lib_ab.py $c 3 diag/lib_pre_edge.so replicat_amd/libreplicat_chunker.so > $out/lib_ab_$c.log 2>&1 || { echo "lib ab $c failed"; tail -5 $out/lib_ab_$c.log; exit 4; }
  tail -1 $out/lib_ab_$c.log
done
echo done
