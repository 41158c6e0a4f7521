# Round 3: what the tile kernel's per-tile exact key costs -- one allocation, the default build
# against one without the exact key (RC_DIAG_NO_EXACT: wrong records, timed only), loaded side by
# side (scripts/lib_ab.py).  profiles/r03/tail/ also has a third build of that run, the exact key
# on the candidate lanes only (an #ifdef since removed).
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/tail
mkdir -p $out
for cfg in 2 3iii; do
  timeout -k 10 300 python -u scripts/lib_ab.py $cfg 6 replicat_amd/libreplicat_chunker.so diag/lib_NOEXACT.so > $out/ab_$cfg.log 2>&1
  rc=$?; echo "ab $cfg rc=$rc"; grep '^{' $out/ab_$cfg.log
  [ $rc -eq 0 ] || exit $rc
done
