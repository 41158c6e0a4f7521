# Round 3: static share with 12-tile units (one allocation, scripts/overlap_ab.py).
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/sched_static
mkdir -p $out
AB_STEPS=20 timeout -k 10 500 python -u scripts/overlap_ab.py 2 4 p32@250:12 p32@0:12 p32@100:12 p32@400:12 p32@250:10 p64@250:12 seq@250:12 seq@100:12 > $out/ab_2.log 2>&1
rc=$?; echo "ab 2 rc=$rc"; grep '^{' $out/ab_2.log
[ $rc -eq 0 ] || exit $rc
AB_STEPS=10 timeout -k 10 500 python -u scripts/overlap_ab.py 3iii 3 seq@250:12 seq@100:12 seq@0:12 > $out/ab_3iii.log 2>&1
rc=$?; echo "ab 3iii rc=$rc"; grep '^{' $out/ab_3iii.log
exit $rc
