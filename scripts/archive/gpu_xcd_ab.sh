# Round 3: one grab counter (diag/lib_ONECTR.so, the build before) against one per XCD (the
# current library), same allocation, both at the default schedule (scripts/lib_ab.py).
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/xcd_ab
mkdir -p $out
for cfg in 2 4 3iii; do
  timeout -k 10 400 python -u scripts/lib_ab.py $cfg 6 replicat_amd/libreplicat_chunker.so diag/lib_ONECTR.so > $out/ab_$cfg.log 2>&1
  rc=$?; echo "ab $cfg rc=$rc"; grep '^{' $out/ab_$cfg.log
  [ $rc -eq 0 ] || exit $rc
done
