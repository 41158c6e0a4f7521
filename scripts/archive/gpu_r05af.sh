# Round 5, pass af: AES-GCM's Horner step with a nibble word's 8 table lookups in flight before
# any is folded (tab_mul_wide).  GCM parity, then config 2's encryption with the previous library
# (diag/lib_gcm_base.so) and this one alternated, three processes each.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05af
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gcm.py > $out/pytest.log 2>&1 || { echo "tests failed"; tail -30 $out/pytest.log; exit 3; }
tail -2 $out/pytest.log
for i in 1 2 3; do
  RC_LIB_PATH=diag/lib_gcm_base.so timeout -k 10 300 python -u scripts/gcm_probe.py > $out/old_$i.log 2>&1 || { echo "old $i failed"; tail -5 $out/old_$i.log; exit 4; }
  echo "old $(tail -1 $out/old_$i.log | cut -c1-330)"
  timeout -k 10 300 python -u scripts/gcm_probe.py > $out/new_$i.log 2>&1 || { echo "new $i failed"; tail -5 $out/new_$i.log; exit 5; }
  echo "new $(tail -1 $out/new_$i.log | cut -c1-330)"
done
echo done
