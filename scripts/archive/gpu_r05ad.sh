# Round 5, pass ad: BLAKE2b quads' LDS blocks at a 160-byte stride (message-word reads no longer
# ~4-way bank conflicts).  Digest / GCM parity, the bank-conflict counter, then config 2's chunk
# digests with the 128-byte-stride library (diag/lib_b2stride128.so) and this one alternated.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05ad
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_digest.py tests/test_gpu_digest_lanes.py tests/test_gpu_gcm.py tests/test_gpu_pipeline.py > $out/pytest.log 2>&1 || { echo "tests failed"; tail -30 $out/pytest.log; exit 3; }
tail -2 $out/pytest.log
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-include-regex "rc_b2_kernel" --output-format csv -d $out/pmc -o run -- python3 scripts/digest_probe.py > $out/pmc.log 2>&1 || { echo "pmc failed"; tail -n 8 $out/pmc.log; exit 4; }
python3 scripts/pmc_by_kernel.py $out/pmc | tee $out/pmc_by_kernel.txt
for i in 1 2 3; do
  RC_LIB_PATH=diag/lib_b2stride128.so timeout -k 10 200 python -u scripts/digest_probe.py > $out/old_$i.log 2>&1 || { echo "old $i failed"; tail -5 $out/old_$i.log; exit 5; }
  echo "old $(tail -1 $out/old_$i.log)"
  timeout -k 10 200 python -u scripts/digest_probe.py > $out/new_$i.log 2>&1 || { echo "new $i failed"; tail -5 $out/new_$i.log; exit 6; }
  echo "new $(tail -1 $out/new_$i.log)"
done
RC_LIB_PATH=diag/lib_b2stride128.so timeout -k 10 200 python -u scripts/digest_probe.py 65536 1 20000 80000 > $out/old_3iii.log 2>&1 || { echo "old 3iii failed"; exit 7; }
echo "old 3iii $(tail -1 $out/old_3iii.log)"
timeout -k 10 200 python -u scripts/digest_probe.py 65536 1 20000 80000 > $out/new_3iii.log 2>&1 || { echo "new 3iii failed"; exit 8; }
echo "new 3iii $(tail -1 $out/new_3iii.log)"
echo done
