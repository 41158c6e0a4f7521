# Round 5, pass n: AES with all four T-tables in LDS (no rot16 per column) -- the cipher's GPU
# parity tests, then the config-2 encrypted-leg probe alternating the previous library
# (diag/lib_gcm_old.so) and this one, two rounds each.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05n
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gcm.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { echo "gcm tests failed"; tail -30 $out/pytest.log; exit 3; }
tail -n 2 $out/pytest.log
for i in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export RC_LIB_PATH=diag/lib_gcm_old.so; else unset RC_LIB_PATH; fi
    timeout -k 10 300 python -u scripts/gcm_probe.py > $out/probe_${v}_$i.log 2>&1 || { echo "probe $v failed"; tail -20 $out/probe_${v}_$i.log; exit 4; }
    echo "$v $i: $(grep -v amdgpu.ids $out/probe_${v}_$i.log | tail -1 | cut -c1-400 | tr '\n' ' ')"
  done
done
echo done
