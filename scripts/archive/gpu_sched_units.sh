# Round 3: dynamic unit size (tiles per grab) at 25 % static, pipelined (224 CUs) and sequential
# (256 CUs) -- one allocation per config, settings alternating (scripts/overlap_ab.py).
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/sched_units
mkdir -p $out
AB_STEPS=20 timeout -k 10 500 python -u scripts/overlap_ab.py 2 4 p32@250:32 p32@250:24 p32@250:16 p32@250:12 p32@250:8 seq@250:32 seq@250:16 seq@250:8 > $out/ab_2.log 2>&1
rc=$?; echo "ab 2 rc=$rc"; grep '^{' $out/ab_2.log
[ $rc -eq 0 ] || exit $rc
AB_STEPS=10 timeout -k 10 500 python -u scripts/overlap_ab.py 4 3 p32@250:32 p32@250:16 p32@250:8 > $out/ab_4.log 2>&1
rc=$?; echo "ab 4 rc=$rc"; grep '^{' $out/ab_4.log
[ $rc -eq 0 ] || exit $rc
AB_STEPS=10 timeout -k 10 500 python -u scripts/overlap_ab.py 3iii 3 seq@250:32 seq@250:16 seq@250:8 > $out/ab_3iii.log 2>&1
rc=$?; echo "ab 3iii rc=$rc"; grep '^{' $out/ab_3iii.log
exit $rc
